// Grouping math on gfx950: cosine-distance dedupe and classification.
//
// remove_dupes_overall 'enc' (src/videotofaces/dupes.py:51-68) computes
//   D = sklearn cosine_distances(X)               (N x N, materialised, + an fp64 N x N tri)
//   D += (1 - tri(N, k=-1)) * 10000 ; mins = D.min(1) ; inds = D.argmin(1)
// i.e. for each face i: min / first argmin over EARLIER faces j < i of clip(1 - <xi,xj>, 0, 2).
// Row 0 has no earlier face: its masked row gives min 10000 at index 0.
//
// The reference's bits (sklearn 1.7.2 on numpy 2.2 + its OpenBLAS 0.3.29 SKYLAKEX; probes in
// scripts/sklearn_cosine_order.py):
//   normalize   xi = X_i / sqrt(np.einsum('ij,ij->i')) (zero norm -> 1; sklearn/preprocessing
//               _data.py normalize -> row_norms), correctly rounded sqrt and division;
//   Gram        X_n @ X_n.T: numpy's matmul sees one buffer times its transpose and calls
//               cblas_ssyrk (then mirrors the triangle).  OpenBLAS's syrk driver splits K into
//               blocks (448, or the two halves (r + 1) / 2 of a remainder r in (448, 896)); each
//               block is one sequential fma chain from 0 in k order and C += block, in order;
//   distance    S *= -1 ; S += 1 ; clip(0, 2)  ==  clip(1 - g, 0, 2).
// Every product x_i[k] x_j[k] is symmetric in (i, j), so lower and upper triangles agree.
// Here: one fused kernel over 128x128 lower-triangle tiles; each K block accumulates from zero
// (fp32 MFMA 16x16x4: an exact fmaf chain in k order, MI355X_MICROARCH.md -- or the VALU fmaf
// kernel when a block boundary is not a multiple of 4) and is added to the running total at
// the block's end; distance + clip + row-min in the epilogue, one 64-bit atomicMin per (row,
// tile) on the key (dist bits << 32 | j): dist >= 0 so float bits order like the floats, and
// ties resolve to the smallest j = numpy's first argmin.  Nothing N x N ever touches HBM.
// classify (grouping.py:50-66): argmin / min over C references of cosine distance, in sklearn's
// bits (k_classify below).
#include <cstdlib>

#include "common.hpp"
#include "sk_order.hpp"

namespace vtf {

typedef __attribute__((ext_vector_type(4))) float f32x4;

// Xn [N][Dp] = X / ||X|| in sklearn normalize's bits (zero norm -> 1), zero-padded to Dp.  One
// wave per row: the row is read coalesced into LDS, lanes 0-3 run numpy einsum's four sequential
// chains over it (sk_order.hpp's order), every lane writes the normalised row coalesced.
// Rows wider than NRM_LDS_D (the four staged rows would pass the 64 KB dynamic-LDS default) are
// read from global memory directly (G): the same chains, the same bits.
constexpr int NRM_W = 4;  // rows (waves) per block
constexpr int NRM_LDS_D = 4096;
template <bool G>
__global__ __launch_bounds__(64 * NRM_W) void k_row_normalize(const float* __restrict__ X, int64_t N, int D, int Dp,
                                                               float* __restrict__ Xn) {
    extern __shared__ float srow[];  // [NRM_W][D] (!G)
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int64_t i = (int64_t)blockIdx.x * NRM_W + w;
    const bool valid = i < N;
    const float* x = X + (valid ? i : 0) * D;
    const float* r = x;
    if (!G) {
        float* rs = srow + w * D;
        if (valid)
            for (int k = lane; k < D; k += 64) rs[k] = x[k];
        __syncthreads();
        r = rs;
    }
    float l = 0.f;  // lane u < 4: numpy's SSE lane u
    if (lane < 4) {
        int t = 0;
        for (; D - t >= 16; t += 16)
            for (int q = 3; q >= 0; q--) {
                const float v = r[t + 4 * q + lane];
                l = __fadd_rn(__fmul_rn(v, v), l);
            }
        for (; t < D; t += 4) {
            const float v = t + lane < D ? r[t + lane] : 0.f;
            l = __fadd_rn(__fmul_rn(v, v), l);
        }
    }
    const float l1 = __shfl(l, 1), l2 = __shfl(l, 2), l3 = __shfl(l, 3);
    float nrm = sqrtf(__fadd_rn(__fadd_rn(__shfl(l, 0), l1), __fadd_rn(l2, l3)));  // correctly rounded
    if (nrm == 0.f) nrm = 1.f;
    if (valid)
        for (int k = lane; k < Dp; k += 64) Xn[i * Dp + k] = k < D ? __fdiv_rn(r[k], nrm) : 0.f;
}
static void row_normalize(const float* X, int64_t N, int D, int Dp, float* Xn, hipStream_t st) {
    if (D <= NRM_LDS_D)
        k_row_normalize<false><<<cdiv(N, NRM_W), 64 * NRM_W, (size_t)NRM_W * D * 4, st>>>(X, N, D, Dp, Xn);
    else
        k_row_normalize<true><<<cdiv(N, NRM_W), 64 * NRM_W, 0, st>>>(X, N, D, Dp, Xn);
}

__global__ void k_init_keys(uint64_t* key, int64_t N) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < N) key[i] = ~0ull;
}

constexpr int CT = 128, CK = 32, CLD = CK + 4;

__device__ inline void tile_pair(int64_t t, int64_t& bi, int64_t& bj) {
    // tile pair from linear index t: bi = floor((sqrt(8t+1)-1)/2), bj = t - bi(bi+1)/2
    bi = (int64_t)((sqrt(8.0 * (double)t + 1.0) - 1.0) * 0.5);
    while ((bi + 1) * (bi + 2) / 2 <= t) bi++;
    while (bi * (bi + 1) / 2 > t) bi--;
    bj = t - bi * (bi + 1) / 2;
}

__device__ inline void row_key_min(uint64_t& best, int width) {
    for (int off = 1; off < width; off <<= 1) {
        uint32_t lo = __shfl_xor((uint32_t)best, off), hi = __shfl_xor((uint32_t)(best >> 32), off);
        uint64_t o = ((uint64_t)hi << 32) | lo;
        best = o < best ? o : best;
    }
}

__device__ inline uint64_t dist_key(float g, int64_t j) {
    float d = __fsub_rn(1.0f, g);
    d = fminf(fmaxf(d, 0.f), 2.f);
    return ((uint64_t)f2u(d) << 32) | (uint64_t)j;
}

// MFMA form; grid.x enumerates lower-triangle tile pairs (bi >= bj).  Requires every K-block
// boundary to be a multiple of 4 (one MFMA step never straddles two blocks).
__global__ __launch_bounds__(256) void k_cos_dedupe(const float* __restrict__ Xn, int64_t N, int D, int Dp,
                                                    int64_t t_base, int64_t row0, uint64_t* __restrict__ key) {
    __shared__ __attribute__((aligned(16))) float As[CT * CLD];
    __shared__ __attribute__((aligned(16))) float Bs[CT * CLD];
    int64_t bi, bj;
    tile_pair(t_base + blockIdx.x, bi, bj);
    const int64_t i0 = bi * CT, j0 = bj * CT;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    f32x4 acc[4][4], tot[4][4];
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
        for (int b = 0; b < 4; b++) acc[a][b] = tot[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    int kb_end = blas_kblock(D, true);
    for (int k0 = 0; k0 < Dp; k0 += CK) {
        // 128 rows x 32 floats per operand = 1024 float4; 4 per thread
#pragma unroll
        for (int r = 0; r < 4; r++) {
            int v = tid + 256 * r;
            int row = v >> 3, kq = (v & 7) * 4;
            f32x4 a = {}, b = {};
            if (i0 + row < N) a = *(const f32x4*)(Xn + (i0 + row) * Dp + k0 + kq);
            if (j0 + row < N) b = *(const f32x4*)(Xn + (j0 + row) * Dp + k0 + kq);
            *(f32x4*)(As + row * CLD + kq) = a;
            *(f32x4*)(Bs + row * CLD + kq) = b;
        }
        __syncthreads();
        const float* Aw = As + (wm * 64 + (lane & 15)) * CLD + (lane >> 4);
        const float* Bw = Bs + (wn * 64 + (lane & 15)) * CLD + (lane >> 4);
#pragma unroll
        for (int ks = 0; ks < CK; ks += 4) {
            if (k0 + ks == kb_end) {  // end of a K block: C += block (uniform branch)
#pragma unroll
                for (int a = 0; a < 4; a++)
#pragma unroll
                    for (int b = 0; b < 4; b++) {
#pragma unroll
                        for (int q = 0; q < 4; q++) tot[a][b][q] = __fadd_rn(tot[a][b][q], acc[a][b][q]);
                        acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
                    }
                kb_end += blas_kblock(D - kb_end, true);
            }
            float af[4], bfr[4];
#pragma unroll
            for (int a = 0; a < 4; a++) af[a] = Aw[a * 16 * CLD + ks];
#pragma unroll
            for (int b = 0; b < 4; b++) bfr[b] = Bw[b * 16 * CLD + ks];
#pragma unroll
            for (int a = 0; a < 4; a++)
#pragma unroll
                for (int b = 0; b < 4; b++)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[a], bfr[b], acc[a][b], 0, 0, 0);
        }
        __syncthreads();
    }
    // epilogue: row i = i0 + wm*64 + a*16 + 4*(lane>>4) + q, col j = j0 + wn*64 + b*16 + (lane&15)
#pragma unroll
    for (int a = 0; a < 4; a++) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            int64_t i = i0 + wm * 64 + a * 16 + 4 * (lane >> 4) + q;
            uint64_t best = ~0ull;
#pragma unroll
            for (int b = 0; b < 4; b++) {
                int64_t j = j0 + wn * 64 + b * 16 + (lane & 15);
                if (i < N && j < i) {
                    uint64_t k = dist_key(__fadd_rn(tot[a][b][q], acc[a][b][q]), j);
                    best = k < best ? k : best;
                }
            }
            row_key_min(best, 16);  // the 16 lanes that share this row (lane & 15 varies)
            if ((lane & 15) == 0 && best != ~0ull) atomicMin((unsigned long long*)&key[i - row0], (unsigned long long)best);
        }
    }
}

// VALU form (any K-block boundary): 16x16 threads, each an 8x8 micro-tile (rows ty*4 + {0..3}
// and 64 + ty*4 + {0..3}, columns likewise by tx), operands k-major in LDS, one fmaf per
// product in k order.
constexpr int VK = 16, VLD = CT + 4;
__global__ __launch_bounds__(256) void k_cos_dedupe_valu(const float* __restrict__ Xn, int64_t N, int D, int Dp,
                                                         int64_t t_base, int64_t row0, uint64_t* __restrict__ key) {
    __shared__ __attribute__((aligned(16))) float As[VK * VLD];
    __shared__ __attribute__((aligned(16))) float Bs[VK * VLD];
    int64_t bi, bj;
    tile_pair(t_base + blockIdx.x, bi, bj);
    const int64_t i0 = bi * CT, j0 = bj * CT;
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    float acc[8][8], tot[8][8];
#pragma unroll
    for (int a = 0; a < 8; a++)
#pragma unroll
        for (int b = 0; b < 8; b++) acc[a][b] = tot[a][b] = 0.f;
    int kb_end = blas_kblock(D, true);
    for (int k0 = 0; k0 < Dp; k0 += VK) {
        // 128 rows x 16 floats per operand = 512 float4; 2 per thread, stored k-major
#pragma unroll
        for (int r = 0; r < 2; r++) {
            int v = tid + 256 * r;
            int row = v >> 2, kq = (v & 3) * 4;
            f32x4 a = {}, b = {};
            if (i0 + row < N) a = *(const f32x4*)(Xn + (i0 + row) * Dp + k0 + kq);
            if (j0 + row < N) b = *(const f32x4*)(Xn + (j0 + row) * Dp + k0 + kq);
#pragma unroll
            for (int u = 0; u < 4; u++) {
                As[(kq + u) * VLD + row] = a[u];
                Bs[(kq + u) * VLD + row] = b[u];
            }
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < VK; kk++) {
            if (k0 + kk == kb_end) {
#pragma unroll
                for (int a = 0; a < 8; a++)
#pragma unroll
                    for (int b = 0; b < 8; b++) {
                        tot[a][b] = __fadd_rn(tot[a][b], acc[a][b]);
                        acc[a][b] = 0.f;
                    }
                kb_end += blas_kblock(D - kb_end, true);
            }
            const f32x4 a0 = *(const f32x4*)(As + kk * VLD + ty * 4), a1 = *(const f32x4*)(As + kk * VLD + 64 + ty * 4);
            const f32x4 b0 = *(const f32x4*)(Bs + kk * VLD + tx * 4), b1 = *(const f32x4*)(Bs + kk * VLD + 64 + tx * 4);
            float av[8] = {a0[0], a0[1], a0[2], a0[3], a1[0], a1[1], a1[2], a1[3]};
            float bv[8] = {b0[0], b0[1], b0[2], b0[3], b1[0], b1[1], b1[2], b1[3]};
#pragma unroll
            for (int a = 0; a < 8; a++)
#pragma unroll
                for (int b = 0; b < 8; b++) acc[a][b] = fmaf(av[a], bv[b], acc[a][b]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int a = 0; a < 8; a++) {
        const int64_t i = i0 + (a >> 2) * 64 + ty * 4 + (a & 3);
        uint64_t best = ~0ull;
#pragma unroll
        for (int b = 0; b < 8; b++) {
            const int64_t j = j0 + (b >> 2) * 64 + tx * 4 + (b & 3);
            if (i < N && j < i) {
                uint64_t k = dist_key(__fadd_rn(tot[a][b], acc[a][b]), j);
                best = k < best ? k : best;
            }
        }
        row_key_min(best, 16);  // lanes with the same ty: 16 consecutive lanes
        if (tx == 0 && best != ~0ull) atomicMin((unsigned long long*)&key[i - row0], (unsigned long long)best);
    }
}

__global__ void k_unpack(const uint64_t* __restrict__ key, int64_t N, float* __restrict__ mn, int64_t* __restrict__ arg) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;  // (row-range-relative index: key, mn and arg all start at the range)
    uint64_t k = key[i];
    if (k == ~0ull) {  // row 0: every entry masked -> 0 + 10000 at j = 0
        mn[i] = 10000.f;
        arg[i] = 0;
    } else {
        mn[i] = __builtin_bit_cast(float, (uint32_t)(k >> 32));
        arg[i] = (int64_t)(uint32_t)k;
    }
}

// ---- classify (grouping.py:50-53): cosine_distances(X, R) in sklearn's bits -------------------
// X_n @ R_n.T is numpy matmul on two buffers (OpenBLAS 0.3.29 SkylakeX kernels; probed by
// absorption and checked bit for bit against sklearn in the survey container: oracle/
// grouping_oracle.c, tests/test_oracle.py::test_classify_restatement_vs_sklearn):
//   CL_BLOCKED  sgemm, blocked kernel: K blocks of gemm's rule (sk_order.hpp), one fmaf chain per
//               block from 0, G += block;
//   CL_SMALL    sgemm small-matrix kernel (N C D <= 1e6, C N <= 1200, D >= 32): 16 lanes over
//               d mod 16, one fmaf chain each; adjacent-pair lane tree, halving tree on the edge
//               block (row >= N - N % 4 and class >= C - C % 4);
//   CL_GEMV     one side a single row: sgemv_t, each output by one of three kernels: 4x4 (8 lanes
//               over d mod 8, fmaf), 4x2 (4 lanes, product then add), 4x1 (8 lanes, product then
//               add); lane trees (l_u + l_{u+4}) then (a0 + a1) + (a2 + a3), resp.
//               (l0 + l1) + (l2 + l3).  Outputs are split over OpenBLAS's threads when D n >=
//               460800 (8 threads in the survey container), 4x4 groups first in every range;
//   CL_DOT      a single row each: sdot, 64 lanes over d mod 64 (8 accumulators of 8 lanes),
//               (((c0 + c1) + (c2 + c3)) + (c4 + c5)) + (c6 + c7), then the 8 lanes as in 4x4.
// Then d = clip(1 - G, 0, 2) (S *= -1; S += 1; np.clip keeps NaN) and numpy's min / first argmin
// (a NaN wins both).
enum { CL_BLOCKED = 1, CL_SMALL = 2, CL_GEMV = 3, CL_DOT = 4 };
// OpenBLAS threads of the sgemv output split: the survey container's 8 (its 8 cores) unless
// VTF_BLAS_THREADS names the reference host's count.  Only CL_GEMV at D n >= 460800 depends on it:
// its bit parity with sklearn assumes that host's thread count
constexpr int CL_BLAS_THREADS = 8;
static int blas_threads() {
    const char* e = std::getenv("VTF_BLAS_THREADS");
    const int v = e ? std::atoi(e) : 0;
    return v >= 1 && v <= 1024 ? v : CL_BLAS_THREADS;
}

__host__ __device__ inline int classify_mode(int64_t N, int64_t C, int64_t D) {
    if (N == 1 && C == 1) return CL_DOT;
    if (N == 1 || C == 1) return CL_GEMV;
    return ((double)N * C * D <= 1e6 && C * N <= 1200 && D >= 32) ? CL_SMALL : CL_BLOCKED;
}

// sgemv_t kernel of output o of n: 0 = 4x4, 1 = 4x2, 2 = 4x1
__device__ inline int gemv_kernel(int64_t o, int64_t n, int64_t D, int threads) {
    const int T = (double)n * D >= 460800.0 ? threads : 1;
    int64_t a = 0;
    for (int t = 0; a < n; t++) {
        int64_t w = T - t > 1 ? (n - a + (T - t) - 1) / (T - t) : n - a;
        w = min(max(w, (int64_t)4), n - a);
        if (o < a + w) {
            const int64_t r = o - a, q = w / 4 * 4;
            if (r < q) return 0;
            return (w & 2) && r < q + 2 ? 1 : 2;
        }
        a += w;
    }
    return 0;
}

constexpr int CL_R = 16, CL_C = 16, CL_K = 64;
template <int MODE>
__global__ __launch_bounds__(256) void k_classify(const float* __restrict__ Xn, const float* __restrict__ Rn, int64_t N,
                                                  int C, int D, int Dp, float* __restrict__ mn,
                                                  int64_t* __restrict__ arg, float* __restrict__ dist, int threads) {
    __shared__ float sX[CL_R][CL_K + 1], sR[CL_C][CL_K + 1];
    __shared__ float sD[CL_R][CL_C];
    const int tid = threadIdx.x, r = tid >> 4, cj = tid & 15;
    const int64_t i0 = (int64_t)blockIdx.x * CL_R, i = i0 + r;
    float best = 0.f;
    int bk = -1;
    for (int c0 = 0; c0 < C; c0 += CL_C) {
        const int c = c0 + cj;
        constexpr int L = MODE == CL_DOT ? 64 : (MODE == CL_SMALL ? 16 : 8);
        float l[L];
#pragma unroll
        for (int u = 0; u < L; u++) l[u] = 0.f;
        float acc = 0.f, tot = 0.f;
        int kb_end = blas_kblock(D, false);
        int gk = 0;  // CL_GEMV: this output's kernel
        if (MODE == CL_GEMV) gk = C == 1 ? gemv_kernel(i, N, D, threads) : gemv_kernel(c, C, D, threads);
        for (int t0 = 0; t0 < Dp; t0 += CL_K) {
            for (int e = tid; e < CL_R * CL_K; e += 256) {  // rows of 64 floats: coalesced
                const int rr = e / CL_K, tt = e % CL_K;
                sX[rr][tt] = i0 + rr < N ? Xn[(i0 + rr) * Dp + t0 + tt] : 0.f;
                sR[rr][tt] = c0 + rr < C ? Rn[(int64_t)(c0 + rr) * Dp + t0 + tt] : 0.f;
            }
            __syncthreads();
            const int tn = min(CL_K, D - t0);
#pragma unroll
            for (int tt = 0; tt < CL_K; tt++) {
                if (tt < tn) {
                    const float a = sX[r][tt], b = sR[cj][tt];
                    if (MODE == CL_BLOCKED) {
                        acc = fmaf(a, b, acc);
                        if (t0 + tt + 1 == kb_end) {  // end of a K block: G += block
                            tot = __fadd_rn(tot, acc);
                            acc = 0.f;
                            kb_end += blas_kblock(D - kb_end, false);
                        }
                    } else if (MODE == CL_GEMV) {
                        if (gk == 0) {
                            l[tt & 7] = fmaf(a, b, l[tt & 7]);
                        } else {
                            const float p = __fmul_rn(a, b);
                            if (gk == 1) l[tt & 3] = __fadd_rn(l[tt & 3], p);
                            else l[tt & 7] = __fadd_rn(l[tt & 7], p);
                        }
                    } else {
                        l[tt % L] = fmaf(a, b, l[tt % L]);
                    }
                }
            }
            __syncthreads();
        }
        float g;
        if (MODE == CL_BLOCKED) {
            g = tot;
        } else if (MODE == CL_SMALL) {
            if (i >= N - N % 4 && c >= C - C % 4) {  // edge block of the C tile: halving tree
#pragma unroll
                for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
                    for (int u = 0; u < w; u++) l[u] = __fadd_rn(l[u], l[u + w]);
            } else {  // adjacent pairs
#pragma unroll
                for (int w = 1; w < 16; w <<= 1)
#pragma unroll
                    for (int u = 0; u < 16; u += 2 * w) l[u] = __fadd_rn(l[u], l[u + w]);
            }
            g = l[0];
        } else {
            float v[8];
            if (MODE == CL_DOT) {
#pragma unroll
                for (int u = 0; u < 8; u++) {
                    const float c01 = __fadd_rn(l[u], l[8 + u]), c23 = __fadd_rn(l[16 + u], l[24 + u]);
                    const float c45 = __fadd_rn(l[32 + u], l[40 + u]), c67 = __fadd_rn(l[48 + u], l[56 + u]);
                    v[u] = __fadd_rn(__fadd_rn(__fadd_rn(c01, c23), c45), c67);
                }
            } else {
#pragma unroll
                for (int u = 0; u < 8; u++) v[u] = l[u];
            }
            if (MODE == CL_GEMV && gk == 1) {
                g = __fadd_rn(__fadd_rn(v[0], v[1]), __fadd_rn(v[2], v[3]));
            } else {
                const float a0 = __fadd_rn(v[0], v[4]), a1 = __fadd_rn(v[1], v[5]);
                const float a2 = __fadd_rn(v[2], v[6]), a3 = __fadd_rn(v[3], v[7]);
                g = __fadd_rn(__fadd_rn(a0, a1), __fadd_rn(a2, a3));
            }
        }
        float d = __fsub_rn(1.0f, g);
        d = d < 0.f ? 0.f : (d > 2.f ? 2.f : d);  // (NaN stays NaN, as np.clip)
        sD[r][cj] = d;
        if (dist && i < N && c < C) dist[i * C + c] = d;  // (the full matrix: classify's CSV log)
        __syncthreads();
        if (cj == 0 && mn) {  // numpy min / first argmin over the row, chunk by chunk in class order
            for (int q = 0; q < CL_C && c0 + q < C; q++) {
                const float v = sD[r][q];
                if (bk < 0 || (best == best && (v != v || v < best))) {
                    best = v;
                    bk = c0 + q;
                }
            }
        }
        __syncthreads();
    }
    if (cj == 0 && i < N && mn) {
        mn[i] = best;
        arg[i] = bk;
    }
}

}  // namespace vtf

using namespace vtf;

extern "C" {

static void cosine_dedupe_rows(const float* d_X, int64_t N, int64_t D, int64_t r0, int64_t r1, float* d_min,
                               int64_t* d_arg, hipStream_t st) {
    VTF_CHECK(d_X && d_min && d_arg && N < (int64_t)1 << 31, VTF_E_ARG, "bad argument");
    VTF_CHECK(0 <= r0 && r0 <= r1 && r1 <= N && r0 % CT == 0 && (r1 % CT == 0 || r1 == N), VTF_E_ARG,
              "row range must be [a, b) with a, b multiples of 128 (or b = N)");
    if (r1 == r0) return;
    StreamScratch sc = stream_scratch(st);
    Arena& ar = *sc.ar;
    int Dp = (int)((D + CK - 1) / CK * CK);
    float* Xn = ar.get<float>(0, N * Dp);
    uint64_t* key = ar.get<uint64_t>(1, r1 - r0);
    // rows r1.. are never read (tiles pair a row block with itself and earlier blocks only)
    row_normalize(d_X, r1, (int)D, Dp, Xn, st);
    k_init_keys<<<cdiv(r1 - r0, 256), 256, 0, st>>>(key, r1 - r0);
    const int64_t b0 = r0 / CT, b1 = (r1 + CT - 1) / CT;
    const int64_t t0 = b0 * (b0 + 1) / 2, t1 = b1 * (b1 + 1) / 2;
    VTF_CHECK(t1 - t0 < (int64_t)1 << 31, VTF_E_LIMIT, "cosine_dedupe: N too large");
    // the MFMA form needs every K-block boundary on a 4-step (one MFMA never spans two blocks)
    bool mfma = true;
    for (int k = blas_kblock((int)D, true); k < D; k += blas_kblock((int)(D - k), true)) mfma &= k % 4 == 0;
    if (const char* e = getenv("VTF_COS_VALU")) mfma &= atoi(e) == 0;
    if (mfma)
        k_cos_dedupe<<<(unsigned)(t1 - t0), 256, 0, st>>>(Xn, N, (int)D, Dp, t0, r0, key);
    else
        k_cos_dedupe_valu<<<(unsigned)(t1 - t0), 256, 0, st>>>(Xn, N, (int)D, Dp, t0, r0, key);
    k_unpack<<<cdiv(r1 - r0, 256), 256, 0, st>>>(key, r1 - r0, d_min, d_arg);
    VTF_HIP(hipGetLastError());
}

int vtf_cosine_dedupe(const float* d_X, int64_t N, int64_t D, float* d_min, int64_t* d_arg, void* hip_stream) {
    return guarded_on(stream_device((hipStream_t)hip_stream), [&] {
        VTF_CHECK(N >= 0 && D > 0, VTF_E_ARG, "bad argument");
        if (N == 0) return;
        cosine_dedupe_rows(d_X, N, D, 0, N, d_min, d_arg, (hipStream_t)hip_stream);
    });
}

int vtf_cosine_dedupe_rows(const float* d_X, int64_t N, int64_t D, int64_t row_begin, int64_t row_end, float* d_min,
                           int64_t* d_arg, void* hip_stream) {
    return guarded_on(stream_device((hipStream_t)hip_stream), [&] {
        VTF_CHECK(N >= 0 && D > 0, VTF_E_ARG, "bad argument");
        if (N == 0) return;
        cosine_dedupe_rows(d_X, N, D, row_begin, row_end, d_min, d_arg, (hipStream_t)hip_stream);
    });
}

static void cosine_classify(const float* d_X, int64_t N, const float* d_R, int64_t C, int64_t D, float* d_min,
                            int64_t* d_arg, float* d_dist, hipStream_t st) {
    VTF_CHECK(N >= 0 && C > 0 && D > 0, VTF_E_ARG, "bad argument");
    if (N == 0) return;
    VTF_CHECK(d_X && d_R && (d_dist || (d_min && d_arg)), VTF_E_ARG, "null argument");
    VTF_CHECK(C < (int64_t)1 << 31 && D < (int64_t)1 << 30, VTF_E_ARG, "bad argument");
    StreamScratch sc = stream_scratch(st);
    Arena& ar = *sc.ar;
    const int Dp = (int)((D + CL_K - 1) / CL_K * CL_K);
    float* Xn = ar.get<float>(2, N * Dp);
    float* Rn = ar.get<float>(3, C * Dp);
    row_normalize(d_X, N, (int)D, Dp, Xn, st);
    row_normalize(d_R, C, (int)D, Dp, Rn, st);
    const unsigned grid = (unsigned)cdiv(N, CL_R);
    const int c = (int)C, d = (int)D, bt = blas_threads();
    switch (classify_mode(N, C, D)) {
        case CL_BLOCKED: k_classify<CL_BLOCKED><<<grid, 256, 0, st>>>(Xn, Rn, N, c, d, Dp, d_min, d_arg, d_dist, bt); break;
        case CL_SMALL: k_classify<CL_SMALL><<<grid, 256, 0, st>>>(Xn, Rn, N, c, d, Dp, d_min, d_arg, d_dist, bt); break;
        case CL_GEMV: k_classify<CL_GEMV><<<grid, 256, 0, st>>>(Xn, Rn, N, c, d, Dp, d_min, d_arg, d_dist, bt); break;
        default: k_classify<CL_DOT><<<grid, 256, 0, st>>>(Xn, Rn, N, c, d, Dp, d_min, d_arg, d_dist, bt); break;
    }
    VTF_HIP(hipGetLastError());
}

int vtf_cosine_classify(const float* d_X, int64_t N, const float* d_R, int64_t C, int64_t D, float* d_min,
                        int64_t* d_arg, void* hip_stream) {
    return guarded_on(stream_device((hipStream_t)hip_stream), [&] {
        VTF_CHECK(d_min && d_arg, VTF_E_ARG, "null argument");
        cosine_classify(d_X, N, d_R, C, D, d_min, d_arg, nullptr, (hipStream_t)hip_stream);
    });
}

int vtf_cosine_distances_xr(const float* d_X, int64_t N, const float* d_R, int64_t C, int64_t D, float* d_dist,
                            void* hip_stream) {
    return guarded_on(stream_device((hipStream_t)hip_stream), [&] {
        VTF_CHECK(d_dist, VTF_E_ARG, "null argument");
        cosine_classify(d_X, N, d_R, C, D, nullptr, nullptr, d_dist, (hipStream_t)hip_stream);
    });
}

}  // extern "C"

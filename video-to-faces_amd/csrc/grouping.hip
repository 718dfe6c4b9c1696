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
// classify (grouping.py:50-66): argmin / min over C references of cosine distance.
#include "common.hpp"
#include "sk_order.hpp"

namespace vtf {

typedef __attribute__((ext_vector_type(4))) float f32x4;

// Xn [N][Dp] = X / ||X|| in sklearn normalize's bits (zero norm -> 1), zero-padded to Dp;
// one thread per row (numpy's einsum order is a 4-lane sequential chain)
__global__ void k_row_normalize(const float* __restrict__ X, int64_t N, int D, int Dp, float* __restrict__ Xn) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    const float* x = X + i * D;
    float nrm = sqrtf(np_einsum_sq(x, D));  // correctly rounded (hipcc's __fsqrt_rn is the 1-ulp v_sqrt_f32)
    if (nrm == 0.f) nrm = 1.f;
    for (int k = 0; k < Dp; k++) Xn[i * Dp + k] = k < D ? __fdiv_rn(x[k], nrm) : 0.f;
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

__global__ void k_classify(const float* __restrict__ Xn, const float* __restrict__ Rn, int64_t N, int C, int Dp,
                           float* __restrict__ mn, int64_t* __restrict__ arg) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    float best = 3.4e38f;
    int bk = 0;
    for (int c = 0; c < C; c++) {
        float s = 0.f;
        for (int k = 0; k < Dp; k++) s = fmaf(Xn[i * Dp + k], Rn[(int64_t)c * Dp + k], s);
        float d = fminf(fmaxf(1.0f - s, 0.f), 2.f);
        if (d < best) {
            best = d;
            bk = c;
        }
    }
    mn[i] = best;
    arg[i] = bk;
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
    k_row_normalize<<<cdiv(r1, 64), 64, 0, st>>>(d_X, r1, (int)D, Dp, Xn);
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

int vtf_cosine_classify(const float* d_X, int64_t N, const float* d_R, int64_t C, int64_t D, float* d_min,
                        int64_t* d_arg, void* hip_stream) {
    return guarded_on(stream_device((hipStream_t)hip_stream), [&] {
        VTF_CHECK(N >= 0 && C > 0 && D > 0, VTF_E_ARG, "bad argument");
        if (N == 0) return;
        VTF_CHECK(d_X && d_R && d_min && d_arg, VTF_E_ARG, "null argument");
        hipStream_t st = (hipStream_t)hip_stream;
        StreamScratch sc = stream_scratch(st);
        Arena& ar = *sc.ar;
        int Dp = (int)((D + CK - 1) / CK * CK);
        float* Xn = ar.get<float>(2, N * Dp);
        float* Rn = ar.get<float>(3, C * Dp);
        k_row_normalize<<<cdiv(N, 64), 64, 0, st>>>(d_X, N, (int)D, Dp, Xn);
        k_row_normalize<<<cdiv(C, 64), 64, 0, st>>>(d_R, C, (int)D, Dp, Rn);
        k_classify<<<cdiv(N, 128), 128, 0, st>>>(Xn, Rn, N, (int)C, Dp, d_min, d_arg);
        VTF_HIP(hipGetLastError());
    });
}

}  // extern "C"

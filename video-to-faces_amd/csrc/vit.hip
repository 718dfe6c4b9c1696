// ViT-B/16 and ViT-L/16 encoders on gfx950 (fp32 MFMA, or fp32-grade split-fp16 MFMA, guarded).
//
// Replaces ViT / AnimeVIT (src/videotofaces/encoders/vit.py:9-146):
//   patch conv 16x16/16 -> [N,64,D]; CLS + pos -> [N,65,D]; depth x pre-LN blocks
//   (LN eps 1e-12 -> fused q|k|v GEMM -> 65-token softmax(q k^T / 8) v per head -> proj +
//   residual -> LN -> fc1 + exact GELU -> fc2 + residual); LN of the CLS row -> [N,D].
// Every GEMM (patch embed as a 16x16 stride-16 conv, q|k|v, proj, fc1, fc2) is the MFMA
// implicit-GEMM kernel (conv.hip) as a 1x1 conv over M = N*65 token rows, with bias /
// residual / GELU fused in the epilogue.  Attention: one workgroup per (image, head) keeps
// Q, K, V (65 x 64 each) and the 65 x 65 scores in LDS; row softmax by wave reductions.
#include <cmath>
#include <cstdlib>
#include <string>
#include <vector>

#include "blob.hpp"
#include "boxes.hpp"
#include "common.hpp"
#include "conv.hpp"
#include "gemm_x3.hpp"

namespace vtf {

constexpr int VT = 65;   // tokens: 64 patches + CLS (img 128, patch 16)
constexpr int VHD = 64;  // head dim (dim // 64 heads)

// x [N,65,D]: row 0 = cls + pos[0], row 1+p = patch[p] + pos[1+p]  (vit.py:96-99)
__global__ void k_vit_tokens(const float* __restrict__ patches, const float* __restrict__ cls,
                             const float* __restrict__ pos, int64_t N, int D, float* __restrict__ x) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N * VT * D) return;
    int d = (int)(i % D);
    int t = (int)((i / D) % VT);
    int64_t n = i / ((int64_t)VT * D);
    float v = t == 0 ? cls[d] : patches[(n * 64 + (t - 1)) * D + d];
    x[i] = v + pos[t * D + d];
}

// LayerNorm over the last dim (eps), rows of length D (D % 256 == 0, D <= 1024) with row stride
// `ld`: one wave per row, 4 rows per workgroup; the row is read once into registers (16-B
// loads), mean and variance are wave reductions over it, then the normalised row is written
constexpr int LN_ROWS = 4;
constexpr int LN_MAXV = 4;  // float4 per lane: D <= 1024
// SP: the normalised rows go out in the split-pair layout of the split-fp16 GEMM (gemm_x3.hpp,
// row stride D * 4 bytes) and an element beyond the fp16 range raises *ovf
template <bool SP = false>
__global__ __launch_bounds__(256) void k_layernorm(const float* __restrict__ x, int64_t rows, int D, int64_t ld,
                                                   const float* __restrict__ g, const float* __restrict__ b, float eps,
                                                   float* __restrict__ y, int64_t ldy, int* __restrict__ ovf = nullptr) {
    const int lane = threadIdx.x & 63;
    const int64_t r = (int64_t)blockIdx.x * LN_ROWS + (threadIdx.x >> 6);
    if (r >= rows) return;
    const int nv = D / 256;  // float4 per lane
    const float4* xr = (const float4*)(x + r * ld);
    float4 v[LN_MAXV];
    float s = 0.f;
#pragma unroll
    for (int j = 0; j < LN_MAXV; j++)
        if (j < nv) {
            v[j] = xr[lane + 64 * j];
            s += (v[j].x + v[j].y) + (v[j].z + v[j].w);
        }
    for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
    const float mean = s / (float)D;
    float q = 0.f;
#pragma unroll
    for (int j = 0; j < LN_MAXV; j++)
        if (j < nv) {
            v[j].x -= mean;
            v[j].y -= mean;
            v[j].z -= mean;
            v[j].w -= mean;
            q = fmaf(v[j].x, v[j].x, q);
            q = fmaf(v[j].y, v[j].y, q);
            q = fmaf(v[j].z, v[j].z, q);
            q = fmaf(v[j].w, v[j].w, q);
        }
    for (int off = 32; off > 0; off >>= 1) q += __shfl_xor(q, off);
    const float rstd = 1.0f / sqrtf(q / (float)D + eps);
    float4* yr = (float4*)(y + r * ldy);
    const float4* g4 = (const float4*)g;
    const float4* b4 = (const float4*)b;
    bool bad = false;
#pragma unroll
    for (int j = 0; j < LN_MAXV; j++)
        if (j < nv) {
            const int c = lane + 64 * j;
            const float4 gg = g4[c], bb = b4[c];
            const float4 o = make_float4(fmaf(v[j].x * rstd, gg.x, bb.x), fmaf(v[j].y * rstd, gg.y, bb.y),
                                         fmaf(v[j].z * rstd, gg.z, bb.z), fmaf(v[j].w * rstd, gg.w, bb.w));
            if constexpr (SP)
                sp_store4((char*)y + r * (int64_t)D * 4, 4 * c, o.x, o.y, o.z, o.w, bad);
            else
                yr[c] = o;
        }
    if constexpr (SP)
        if (__ballot(bad) && lane == 0) atomicOr(ovf, 1);
}

// qkv [N,65,3D] (q | k | v, head-major inside each) -> out [N,65,D]; one workgroup per (n, head).
// SP: out in the split-pair layout of the split-fp16 GEMM (proj's operand), range flag *ovf
template <bool SP = false>
__global__ __launch_bounds__(256) void k_vit_attention(const float* __restrict__ qkv, int64_t N, int D, int heads,
                                                       float* __restrict__ out, int* __restrict__ ovf = nullptr) {
    __shared__ __attribute__((aligned(16))) float V[VT * VHD];  // 16-B rows: float4 reads in P V
    __shared__ float Q[VT * (VHD + 1)], K[VT * (VHD + 1)], S[VT * 68];
    const int64_t n = blockIdx.x / heads;
    const int h = blockIdx.x % heads;
    const int tid = threadIdx.x;
    const float* base = qkv + n * VT * 3 * D + h * VHD;
    // 16-B loads (16 per 64-wide head row); Q/K rows are padded to 65 floats in LDS, so their
    // four lanes are stored one by one
    for (int i = tid; i < VT * VHD / 4; i += 256) {
        const int t = i / (VHD / 4), d = 4 * (i % (VHD / 4));
        const float* row = base + (int64_t)t * 3 * D + d;
        const float4 q = *(const float4*)row, k = *(const float4*)(row + D), v = *(const float4*)(row + 2 * D);
        float* qd = Q + t * (VHD + 1) + d;
        float* kd = K + t * (VHD + 1) + d;
        qd[0] = q.x, qd[1] = q.y, qd[2] = q.z, qd[3] = q.w;
        kd[0] = k.x, kd[1] = k.y, kd[2] = k.z, kd[3] = k.w;
        *(float4*)(V + t * VHD + d) = v;
    }
    __syncthreads();
    // scores = q k^T / sqrt(64)  (vit.py:24; division by 8 is exact as * 0.125).  65 = 13 x 5:
    // each of 169 threads keeps a 5 x 5 block of scores in registers (10 LDS reads per 25 FMAs
    // instead of 2 per FMA); every score still accumulates d = 0..63 in order (same bits)
    if (tid < 169) {
        const int a0 = 5 * (tid / 13), c0 = 5 * (tid % 13);
        float acc[5][5];
#pragma unroll
        for (int i = 0; i < 5; i++)
#pragma unroll
            for (int j = 0; j < 5; j++) acc[i][j] = 0.f;
#pragma unroll 4
        for (int d = 0; d < VHD; d++) {
            float q[5], k[5];
#pragma unroll
            for (int i = 0; i < 5; i++) q[i] = Q[(a0 + i) * (VHD + 1) + d];
#pragma unroll
            for (int j = 0; j < 5; j++) k[j] = K[(c0 + j) * (VHD + 1) + d];
#pragma unroll
            for (int i = 0; i < 5; i++)
#pragma unroll
                for (int j = 0; j < 5; j++) acc[i][j] = fmaf(q[i], k[j], acc[i][j]);
        }
#pragma unroll
        for (int i = 0; i < 5; i++)
#pragma unroll
            for (int j = 0; j < 5; j++) S[(a0 + i) * 68 + c0 + j] = acc[i][j] * 0.125f;
    }
    __syncthreads();
    // row softmax: one wave per row (65 entries -> lanes 0..63 + lane 0 takes the 65th)
    const int lane = tid & 63, wave = tid >> 6;
    for (int a = wave; a < VT; a += 4) {
        float v0 = S[a * 68 + lane];
        float v1 = lane == 0 ? S[a * 68 + 64] : -INFINITY;
        float m = fmaxf(v0, v1);
        for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
        float e0 = expf(v0 - m), e1 = lane == 0 ? expf(v1 - m) : 0.f;
        float s = e0 + e1;
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
        float inv = 1.0f / s;
        S[a * 68 + lane] = e0 * inv;
        if (lane == 0) S[a * 68 + 64] = e1 * inv;
    }
    __syncthreads();
    // out = scores @ v, written back head-major: [N,65,D] feature h*64 + d.  208 threads, each a
    // 5-row x 4-feature block (S broadcast reads, one 16-B V read per c); c = 0..64 in order
    float* ob = out + n * VT * D + h * VHD;
    if (tid < 208) {
        const int a0 = 5 * (tid / 16), d0 = 4 * (tid % 16);
        float acc[5][4];
#pragma unroll
        for (int i = 0; i < 5; i++)
#pragma unroll
            for (int j = 0; j < 4; j++) acc[i][j] = 0.f;
#pragma unroll 5
        for (int c = 0; c < VT; c++) {
            const float4 v = *(const float4*)(V + c * VHD + d0);
#pragma unroll
            for (int i = 0; i < 5; i++) {
                const float sc = S[(a0 + i) * 68 + c];
                acc[i][0] = fmaf(sc, v.x, acc[i][0]);
                acc[i][1] = fmaf(sc, v.y, acc[i][1]);
                acc[i][2] = fmaf(sc, v.z, acc[i][2]);
                acc[i][3] = fmaf(sc, v.w, acc[i][3]);
            }
        }
        bool bad = false;
#pragma unroll
        for (int i = 0; i < 5; i++) {
            if constexpr (SP)
                sp_store4((char*)out + (n * VT + a0 + i) * (int64_t)D * 4, h * VHD + d0, acc[i][0], acc[i][1], acc[i][2],
                          acc[i][3], bad);
            else
                *(float4*)(ob + (int64_t)(a0 + i) * D + d0) = make_float4(acc[i][0], acc[i][1], acc[i][2], acc[i][3]);
        }
        if constexpr (SP)
            if (__ballot(bad) && (tid & 63) == 0) atomicOr(ovf, 1);
    }
}

// The same attention on the fp32 matrix cores (v_mfma_f32_16x16x4_f32: exact fp32 products,
// fp32 accumulation in the MFMA's order), used by the split-fp16 mode: q k^T as 5 x 5 blocks
// of 16 x 16 over d = 0..63 (rows 65..79 zero), the row softmax exactly as k_vit_attention, and
// P V as 5 x 4 blocks over c = 0..79 (P columns 65..79 zeroed).  LDS: Q | K (reused for the
// scores, then for the output tile) and V: 65 KB, two workgroups per CU.
constexpr int AP = 80;        // tokens padded to 5 x 16
constexpr int AQ = VHD + 4;   // Q / K / V / O row stride (floats)
constexpr int AS = AP + 4;    // score row stride
template <bool SP>
__global__ __launch_bounds__(256, 2) void k_vit_attention_mfma(const float* __restrict__ qkv, int64_t N, int D, int heads,
                                                               float* __restrict__ out, int* __restrict__ ovf) {
    typedef __attribute__((ext_vector_type(4))) float f4;
    __shared__ __attribute__((aligned(16))) float sm[2 * AP * AQ + AP * AQ];
    float* Q = sm;
    float* K = sm + AP * AQ;
    float* V = sm + 2 * AP * AQ;
    float* S = sm;  // scores / probabilities [AP][AS] over Q | K once q k^T is in registers
    const int64_t n = blockIdx.x / heads;
    const int h = blockIdx.x % heads;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lk = lane >> 4;
    const float* base = qkv + n * VT * 3 * D + h * VHD;
    for (int i = tid; i < AP * VHD / 4; i += 256) {
        const int t = i / (VHD / 4), d = 4 * (i % (VHD / 4));
        f4 q = {0.f, 0.f, 0.f, 0.f}, k = q, v = q;
        if (t < VT) {
            const float* row = base + (int64_t)t * 3 * D + d;
            q = *(const f4*)row;
            k = *(const f4*)(row + D);
            v = *(const f4*)(row + 2 * D);
        }
        *(f4*)(Q + t * AQ + d) = q;
        *(f4*)(K + t * AQ + d) = k;
        *(f4*)(V + t * AQ + d) = v;
    }
    __syncthreads();
    // scores: 25 blocks, wave w takes blocks w, w + 4, ...
    f4 sc[7];
#pragma unroll
    for (int u = 0; u < 7; u++) {
        const int b = wave + 4 * u;
        sc[u] = f4{0.f, 0.f, 0.f, 0.f};
        if (b < 25) {
            const float* qa = Q + ((b / 5) * 16 + lr) * AQ + lk;
            const float* kb = K + ((b % 5) * 16 + lr) * AQ + lk;
#pragma unroll
            for (int ks = 0; ks < VHD; ks += 4) sc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(qa[ks], kb[ks], sc[u], 0, 0, 0);
        }
    }
    __syncthreads();  // Q and K are dead: the scores go over them
#pragma unroll
    for (int u = 0; u < 7; u++) {
        const int b = wave + 4 * u;
        if (b < 25)
#pragma unroll
            for (int i = 0; i < 4; i++) S[((b / 5) * 16 + 4 * lk + i) * AS + (b % 5) * 16 + lr] = sc[u][i] * 0.125f;
    }
    __syncthreads();
    // row softmax over the 65 scores (as k_vit_attention); P columns 65..79 zeroed
    for (int a = wave; a < VT; a += 4) {
        float v0 = S[a * AS + lane];
        float v1 = lane == 0 ? S[a * AS + 64] : -INFINITY;
        float m = fmaxf(v0, v1);
        for (int off = 32; off > 0; off >>= 1) m = fmaxf(m, __shfl_xor(m, off));
        float e0 = expf(v0 - m), e1 = lane == 0 ? expf(v1 - m) : 0.f;
        float s = e0 + e1;
        for (int off = 32; off > 0; off >>= 1) s += __shfl_xor(s, off);
        float inv = 1.0f / s;
        S[a * AS + lane] = e0 * inv;
        if (lane == 0) S[a * AS + 64] = e1 * inv;
        if (lane < AP - VT) S[a * AS + VT + lane] = 0.f;
    }
    __syncthreads();
    // out = P V: 20 blocks (5 row x 4 feature blocks), wave w takes blocks w, w + 4, ...
    f4 oc[5];
#pragma unroll
    for (int u = 0; u < 5; u++) {
        const int b = wave + 4 * u;
        oc[u] = f4{0.f, 0.f, 0.f, 0.f};
        const float* pa = S + ((b >> 2) * 16 + lr) * AS + lk;
        const float* vb = V + lk * AQ + (b & 3) * 16 + lr;
#pragma unroll
        for (int ks = 0; ks < AP; ks += 4) oc[u] = __builtin_amdgcn_mfma_f32_16x16x4f32(pa[ks], vb[ks * AQ], oc[u], 0, 0, 0);
    }
    __syncthreads();  // P is dead: the output tile goes over it
    float* O = sm;
#pragma unroll
    for (int u = 0; u < 5; u++) {
        const int b = wave + 4 * u;
#pragma unroll
        for (int i = 0; i < 4; i++) O[((b >> 2) * 16 + 4 * lk + i) * AQ + (b & 3) * 16 + lr] = oc[u][i];
    }
    __syncthreads();
    bool bad = false;
    for (int i = tid; i < VT * VHD / 4; i += 256) {
        const int t = i / (VHD / 4), d = 4 * (i % (VHD / 4));
        const f4 o = *(const f4*)(O + t * AQ + d);
        if constexpr (SP)
            sp_store4((char*)out + (n * VT + t) * (int64_t)D * 4, h * VHD + d, o[0], o[1], o[2], o[3], bad);
        else
            *(f4*)(out + (n * VT + t) * (int64_t)D + h * VHD + d) = o;
    }
    if constexpr (SP)
        if (__ballot(bad) && lane == 0) atomicOr(ovf, 1);
}

// The split mode's default attention: fp32-grade products on the fp16 matrix cores
// (v_mfma_f32_16x16x32_f16, x0 y0 + 2^-11 (x0 y1 + x1 y0) as k_gemm_x3) with q|k|v read in the
// split-pair layout the q|k|v GEMM writes.  Computed transposed, S^T = K Q^T, so that each lane
// owns one query column: the softmax over the keys is a register reduction plus two lane
// shuffles, and P^T goes from the accumulators straight into the B operand of O^T = V^T P^T
// (the accumulator-as-operand map: element j of lane group g is key 32s + 4g + (j & 3) +
// 16 (j >> 2)); V^T's fragments are transposed LDS reads (ds_read_b64_tr_b16) of V's row-major
// planes.  One workgroup of 5 waves per (image, head), wave w = queries 16w..16w+15 (wave 4:
// query 64 only).  Q goes global -> registers; K and V planes in LDS: 2 x 2 x 80 rows x 160 B
// = 51 KB (row stride 160 B: conflict-free row and transposed reads), 3 workgroups per CU.
// ds_read_b64_tr_b16: lane 4q + p of each 16-lane group addresses row q, columns 4p..4p+3 of a
// 4 x 16 block of 16-bit elements; lane i receives column i (row q in element q).  EXEC all ones.
__device__ inline __attribute__((ext_vector_type(4))) _Float16 lds_tr16(const _Float16* p) {
    typedef __attribute__((__vector_size__(4 * sizeof(__fp16)))) __fp16 fp16x4;
    const fp16x4 r = __builtin_amdgcn_ds_read_tr16_b64_v4f16((__attribute__((address_space(3))) fp16x4*)(p));
    return __builtin_bit_cast(__attribute__((ext_vector_type(4))) _Float16, r);
}
constexpr int XR = 80;   // LDS rows (keys 65..79 zero)
constexpr int XRS = 80;  // plane row stride in halves (160 B)
__global__ __launch_bounds__(320) void k_vit_attention_x3(const void* __restrict__ qkv, int64_t N, int D, int heads,
                                                          void* __restrict__ out, int* __restrict__ ovf) {
    typedef __attribute__((ext_vector_type(4))) float f4;
    typedef __attribute__((ext_vector_type(8))) _Float16 h8;
    typedef __attribute__((ext_vector_type(4))) _Float16 h4;
    typedef __attribute__((ext_vector_type(4))) int i4;
    __shared__ __attribute__((aligned(16))) _Float16 sm[4 * XR * XRS];  // K0 | K1 | V0 | V1
    const int64_t n = blockIdx.x / heads;
    const int h = blockIdx.x % heads;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, g = lane >> 4;
    const int64_t rowb = (int64_t)3 * D * 4;  // SP row bytes (4 per element)
    const char* base = (const char*)qkv + n * VT * rowb + (int64_t)h * VHD * 4;
    // K / V pieces: 2 operands x 65 rows x 16 (8 chunks x 2 planes) x 16 B
    constexpr int NP = 2 * VT * 16;
    constexpr int PPT = (NP + 319) / 320;
    i4 pc[PPT];
#pragma unroll
    for (int u = 0; u < PPT; u++) {
        const int i = tid + 320 * u;
        if (i < NP) {
            const int op = i / (VT * 16), r = (i / 16) % VT, q = i % 16;
            pc[u] = *(const i4*)(base + r * rowb + (int64_t)(op + 1) * D * 4 + q * 16);
        }
    }
    // this wave's queries as B fragments of S^T: k-step s = dims 32s..32s+31, lane group g takes
    // chunk 4s + g (x0 plane, x1 plane); queries past 64 read row 64 (columns never stored)
    const int t = min(16 * wave + lr, VT - 1);
    h8 q0[2], q1[2];
#pragma unroll
    for (int s = 0; s < 2; s++) {
        const char* p = base + t * rowb + (4 * s + g) * 32;
        q0[s] = *(const h8*)p;
        q1[s] = *(const h8*)(p + 16);
    }
    // rows 65..79 of the four planes zeroed (P^T is 0 there; V must be finite)
    for (int i = tid; i < 4 * (XR - VT) * XRS / 8; i += 320) {
        const int pl = i / ((XR - VT) * XRS / 8), o = i % ((XR - VT) * XRS / 8);
        *(i4*)(sm + pl * XR * XRS + VT * XRS + 8 * o) = i4{0, 0, 0, 0};
    }
#pragma unroll
    for (int u = 0; u < PPT; u++) {
        const int i = tid + 320 * u;
        if (i < NP) {
            const int op = i / (VT * 16), r = (i / 16) % VT, q = i % 16;
            // chunk q >> 1 (elements 8j..8j+7), plane q & 1
            *(i4*)(sm + (2 * op + (q & 1)) * XR * XRS + r * XRS + 8 * (q >> 1)) = pc[u];
        }
    }
    __syncthreads();
    const _Float16* K0 = sm;
    const _Float16* K1 = sm + XR * XRS;
    const _Float16* V0 = sm + 2 * XR * XRS;
    const _Float16* V1 = sm + 3 * XR * XRS;
    // S^T blocks: keys 16cb..16cb+15 x this wave's 16 queries
    f4 sc[5];
#pragma unroll
    for (int cb = 0; cb < 5; cb++) {
        f4 a = {0.f, 0.f, 0.f, 0.f}, ax = a;
#pragma unroll
        for (int s = 0; s < 2; s++) {
            const int o = (16 * cb + lr) * XRS + 32 * s + 8 * g;
            const h8 k0 = *(const h8*)(K0 + o), k1 = *(const h8*)(K1 + o);
            a = __builtin_amdgcn_mfma_f32_16x16x32_f16(k0, q0[s], a, 0, 0, 0);
            ax = __builtin_amdgcn_mfma_f32_16x16x32_f16(k0, q1[s], ax, 0, 0, 0);
            ax = __builtin_amdgcn_mfma_f32_16x16x32_f16(k1, q0[s], ax, 0, 0, 0);
        }
        sc[cb] = (a + ax * 0.00048828125f) * 0.125f;  // / sqrt(64) (vit.py:24)
    }
    // column softmax over the 65 keys: lane holds keys 16cb + 4g + i of query column lr
    float m = -INFINITY;
#pragma unroll
    for (int cb = 0; cb < 5; cb++)
#pragma unroll
        for (int i = 0; i < 4; i++)
            if (cb < 4 || (g == 0 && i == 0)) m = fmaxf(m, sc[cb][i]);
    m = fmaxf(m, __shfl_xor(m, 16));
    m = fmaxf(m, __shfl_xor(m, 32));
    float sum = 0.f;
#pragma unroll
    for (int cb = 0; cb < 5; cb++)
#pragma unroll
        for (int i = 0; i < 4; i++) {
            const float e = (cb < 4 || (g == 0 && i == 0)) ? expf(sc[cb][i] - m) : 0.f;
            sc[cb][i] = e;
            sum += e;
        }
    sum += __shfl_xor(sum, 16);
    sum += __shfl_xor(sum, 32);
    const float inv = 1.0f / sum;
    // P^T split into B fragments: k-step s2 = key tiles 2 s2 (elements 0..3) and 2 s2 + 1 (4..7)
    h8 p0[3], p1[3];
#pragma unroll
    for (int s2 = 0; s2 < 3; s2++)
#pragma unroll
        for (int j = 0; j < 8; j++) {
            const int cb = 2 * s2 + (j >> 2);
            const float v = cb < 5 ? sc[cb][j & 3] * inv : 0.f;
            const _Float16 x0 = (_Float16)v;
            p0[s2][j] = x0;
            p1[s2][j] = (_Float16)((v - (float)x0) * 2048.f);
        }
    // O^T blocks: dims 16db..16db+15 x this wave's queries; A = V^T by transposed reads: lane
    // 4q + p of group g addresses key row 32 s2 + 4g (+16) + q, dims 16db + 4p..4p+3
    const int qq = lr >> 2, pp = lr & 3;
    bool bad = false;
#pragma unroll
    for (int db = 0; db < 4; db++) {
        f4 a = {0.f, 0.f, 0.f, 0.f}, ax = a;
#pragma unroll
        for (int s2 = 0; s2 < 3; s2++) {
            const int o = (32 * s2 + 4 * g + qq) * XRS + 16 * db + 4 * pp;
            h4 v0a = lds_tr16((V0 + o));
            h4 v1a = lds_tr16((V1 + o));
            h4 v0b = v0a, v1b = v1a;  // keys 80..95 (P^T = 0 there): any finite values
            if (s2 < 2) {
                v0b = lds_tr16((V0 + o + 16 * XRS));
                v1b = lds_tr16((V1 + o + 16 * XRS));
            }
            const h8 v0 = __builtin_shufflevector(v0a, v0b, 0, 1, 2, 3, 4, 5, 6, 7);
            const h8 v1 = __builtin_shufflevector(v1a, v1b, 0, 1, 2, 3, 4, 5, 6, 7);
            a = __builtin_amdgcn_mfma_f32_16x16x32_f16(v0, p0[s2], a, 0, 0, 0);
            ax = __builtin_amdgcn_mfma_f32_16x16x32_f16(v0, p1[s2], ax, 0, 0, 0);
            ax = __builtin_amdgcn_mfma_f32_16x16x32_f16(v1, p0[s2], ax, 0, 0, 0);
        }
        const f4 o = a + ax * 0.00048828125f;  // O[query 16w + lr][dims 16db + 4g .. +3]
        const int tq = 16 * wave + lr;
        if (tq < VT)
            sp_store4((char*)out + (n * VT + tq) * (int64_t)D * 4, h * VHD + 16 * db + 4 * g, o[0], o[1], o[2], o[3],
                      bad);
    }
    if (__ballot(bad) && lane == 0) atomicOr(ovf, 1);
}

struct Lin {
    const float *w, *b;  // [out][in], [out]
    int in, out;
    const void* sp;      // the weights split once into the SP layout (split-fp16 GEMM), or null
};

struct Vit {
    int device = 0, D = 768, depth = 12, heads = 12;
    // GEMM operand mode: 0 fp32 MFMA; 2 split-fp16 (fp32-grade products on the fp16 matrix
    // cores, conv.hip f16x) guarded by the device overflow flag -> the forward re-runs in fp32
    int xmode = 0, cur_x = 0;
    // split mode on pre-split operands (gemm_x3.hip) when every weight is inside the fp16 range;
    // VTF_VIT_GEMM=conv keeps k_conv's staging-split mode (A/B timing, bit-identical results)
    bool sp_ok = false;
    // split-mode attention: 2 split-fp16 MFMA on split q|k|v (default), 1 fp32 MFMA
    // (VTF_VIT_ATTN=mfma32), 0 the VALU kernel (VTF_VIT_ATTN=valu); 1 and 0 read fp32 q|k|v
    int attn = 2;
    int* d_ovf = nullptr;
    hipStream_t st = 0;
    const float *cls = nullptr, *pos = nullptr, *pw = nullptr, *pb = nullptr;  // patch conv [D][16][16][8]
    struct Block {
        const float *n1w, *n1b, *n2w, *n2b;
        Lin qkv, proj, fc1, fc2;
    };
    std::vector<Block> blocks;
    const float *nw = nullptr, *nb = nullptr;
    std::vector<void*> allocs;
    Arena ar;
    ~Vit() {
        for (void* p : allocs) (void)hipFree(p);
        if (d_ovf) (void)hipFree(d_ovf);
    }
    const void* up_sp(const std::vector<float>& v, int rows, int K) {
        std::vector<uint16_t> h((size_t)rows * K * 2);
        if (!split_rows_host(v.data(), rows, K, h.data())) return nullptr;
        void* p = nullptr;
        VTF_HIP(hipMalloc(&p, h.size() * 2));
        VTF_HIP(hipMemcpy(p, h.data(), h.size() * 2, hipMemcpyHostToDevice));
        allocs.push_back(p);
        return p;
    }
    const float* up(const std::vector<float>& v) {
        void* p = nullptr;
        VTF_HIP(hipMalloc(&p, v.size() * 4 + 16));
        VTF_HIP(hipMemcpy(p, v.data(), v.size() * 4, hipMemcpyHostToDevice));
        allocs.push_back(p);
        return (const float*)p;
    }
};

static void vit_build(Vit& V, const float* params, int64_t n_params) {
    const int D = V.D;
    int64_t src = 0;
    auto take = [&](int64_t n) {
        VTF_CHECK(src + n <= n_params, VTF_E_ARG, "vit: parameter buffer too small");
        std::vector<float> v(params + src, params + src + n);
        src += n;
        return v;
    };
    V.cls = V.up(take(D));
    V.pos = V.up(take((int64_t)VT * D));
    {
        std::vector<float> w = take((int64_t)D * 3 * 256), wt((size_t)D * 256 * 8, 0.f);
        for (int o = 0; o < D; o++)
            for (int c = 0; c < 3; c++)
                for (int y = 0; y < 16; y++)
                    for (int x = 0; x < 16; x++)
                        wt[(((size_t)o * 16 + y) * 16 + x) * 8 + c] = w[(((size_t)o * 3 + c) * 16 + y) * 16 + x];
        V.pw = V.up(wt);
        V.pb = V.up(take(D));
    }
    for (int l = 0; l < V.depth; l++) {
        Vit::Block B{};
        B.n1w = V.up(take(D));
        B.n1b = V.up(take(D));
        std::vector<float> qw = take((int64_t)D * D), qb = take(D), kw = take((int64_t)D * D), kb = take(D),
                           vw = take((int64_t)D * D), vb = take(D);
        std::vector<float> w(qw);
        w.insert(w.end(), kw.begin(), kw.end());
        w.insert(w.end(), vw.begin(), vw.end());
        std::vector<float> b(qb);
        b.insert(b.end(), kb.begin(), kb.end());
        b.insert(b.end(), vb.begin(), vb.end());
        B.qkv = Lin{V.up(w), V.up(b), D, 3 * D, V.up_sp(w, 3 * D, D)};
        { auto pw = take((int64_t)D * D); auto pb = take(D); B.proj = Lin{V.up(pw), V.up(pb), D, D, V.up_sp(pw, D, D)}; }
        B.n2w = V.up(take(D));
        B.n2b = V.up(take(D));
        { auto w1 = take((int64_t)4 * D * D); auto b1 = take(4 * D); B.fc1 = Lin{V.up(w1), V.up(b1), D, 4 * D, V.up_sp(w1, 4 * D, D)}; }
        { auto w2 = take((int64_t)4 * D * D); auto b2 = take(D); B.fc2 = Lin{V.up(w2), V.up(b2), 4 * D, D, V.up_sp(w2, D, 4 * D)}; }
        V.blocks.push_back(B);
    }
    const char* ae = std::getenv("VTF_VIT_ATTN");
    V.attn = !ae ? 2 : std::string(ae) == "valu" ? 0 : std::string(ae) == "mfma32" ? 1 : 2;
    const char* ge = std::getenv("VTF_VIT_GEMM");
    V.sp_ok = !(ge && std::string(ge) == "conv");
    for (const auto& B : V.blocks) V.sp_ok = V.sp_ok && B.qkv.sp && B.proj.sp && B.fc1.sp && B.fc2.sp;
    V.nw = V.up(take(D));
    V.nb = V.up(take(D));
    VTF_CHECK(src == n_params, VTF_E_ARG, "vit: parameter count mismatch");
}

// y[M,out] = x[M,in] W^T + b (+ res) (+ GELU): a 1x1 conv over M rows on the MFMA kernel
static void linear(Vit& V, const Lin& L, const float* x, int64_t M, float* y, const float* res, bool gelu) {
    ConvParams p{};
    p.in = x;
    p.w = L.w;
    p.out = y;
    p.bias = L.b;
    p.res = res;
    p.res_cstride = L.out;
    p.scale = 1.f;
    p.gelu = gelu;
    p.N = (int)M;
    p.H = p.W = p.OH = p.OW = 1;
    p.Cin = L.in;
    p.KH = p.KW = 1;
    p.sh = p.sw = 1;
    p.Cout = L.out;
    p.K = L.in;
    p.M = M;
    p.out_cstride = L.out;
    p.f16x = V.cur_x != 0;
    p.ovf = V.cur_x ? V.d_ovf : nullptr;
    launch_conv(p, false, V.st);
}

// y[M,out] = x W^T + b (+ res) (+ GELU) on pre-split operands: x SP [M][in] -> y fp32 or SP
static void linear_sp(Vit& V, const Lin& L, const void* x, int64_t M, void* y, bool y_sp, const float* res, bool gelu) {
    GemmX3Params p{};
    p.a = x;
    p.b = L.sp;
    p.out = y;
    p.bias = L.b;
    p.res = res;
    p.ldr = L.out;
    p.ovf = V.d_ovf;
    p.M = M;
    p.N = L.out;
    p.K = L.in;
    p.ldo = L.out;
    p.gelu = gelu;
    p.out_sp = y_sp;
    launch_gemm_x3(p, V.st);
}

static void vit_forward(Vit& V, const float* x_nhwc8, int64_t N, float* emb) {
    const int D = V.D;
    const int64_t M = N * VT;
    float* patches = V.ar.get<float>(0, N * 64 * D);
    float* X = V.ar.get<float>(1, M * D);
    float* Hn = V.ar.get<float>(2, M * D);
    float* QKV = V.ar.get<float>(3, M * 3 * D);
    float* A = V.ar.get<float>(4, M * D);
    float* F = V.ar.get<float>(5, M * 4 * D);
    // patch embedding: Conv2d(3, D, 16, stride 16) (vit.py:88,94)
    ConvParams p{};
    p.in = x_nhwc8;
    p.w = V.pw;
    p.out = patches;
    p.bias = V.pb;
    p.scale = 1.f;
    p.N = (int)N;
    p.H = p.W = 128;
    p.Cin = 8;
    p.KH = p.KW = 16;
    p.sh = p.sw = 16;
    p.OH = p.OW = 8;
    p.Cout = D;
    p.K = 16 * 16 * 8;
    p.M = N * 64;
    p.out_cstride = D;
    p.f16x = V.cur_x != 0;
    p.ovf = V.cur_x ? V.d_ovf : nullptr;
    launch_conv(p, false, V.st);
    k_vit_tokens<<<cdiv(M * D, 256), 256, 0, V.st>>>(patches, V.cls, V.pos, N, D, X);
    if (V.cur_x && V.sp_ok) {
        // split mode on pre-split operands: LayerNorm, attention and fc1 write the GEMM operands
        // split (SP), the residual stream X and q|k|v stay fp32; same bits as the k_conv split mode
        const unsigned lg = (unsigned)cdiv(M, LN_ROWS);
        for (const auto& B : V.blocks) {
            k_layernorm<true><<<lg, 256, 0, V.st>>>(X, M, D, D, B.n1w, B.n1b, 1e-12f, Hn, D, V.d_ovf);
            linear_sp(V, B.qkv, Hn, M, QKV, V.attn == 2, nullptr, false);
            if (V.attn == 2)
                k_vit_attention_x3<<<(unsigned)(N * V.heads), 320, 0, V.st>>>(QKV, N, D, V.heads, A, V.d_ovf);
            else if (V.attn == 1)
                k_vit_attention_mfma<true><<<(unsigned)(N * V.heads), 256, 0, V.st>>>(QKV, N, D, V.heads, A, V.d_ovf);
            else
                k_vit_attention<true><<<(unsigned)(N * V.heads), 256, 0, V.st>>>(QKV, N, D, V.heads, A, V.d_ovf);
            linear_sp(V, B.proj, A, M, Hn, false, X, false);  // x + proj(attn)
            std::swap(X, Hn);
            k_layernorm<true><<<lg, 256, 0, V.st>>>(X, M, D, D, B.n2w, B.n2b, 1e-12f, A, D, V.d_ovf);
            linear_sp(V, B.fc1, A, M, F, true, nullptr, true);
            linear_sp(V, B.fc2, F, M, Hn, false, X, false);  // x + fc2(gelu(fc1(...)))
            std::swap(X, Hn);
        }
        k_layernorm<<<(unsigned)cdiv(N, LN_ROWS), 256, 0, V.st>>>(X, N, D, (int64_t)VT * D, V.nw, V.nb, 1e-12f, emb, D);
        return;
    }
    for (const auto& B : V.blocks) {
        k_layernorm<<<(unsigned)cdiv(M, LN_ROWS), 256, 0, V.st>>>(X, M, D, D, B.n1w, B.n1b, 1e-12f, Hn, D);
        linear(V, B.qkv, Hn, M, QKV, nullptr, false);
        k_vit_attention<<<(unsigned)(N * V.heads), 256, 0, V.st>>>(QKV, N, D, V.heads, A);
        linear(V, B.proj, A, M, Hn, X, false);  // x + proj(attn)
        std::swap(X, Hn);
        k_layernorm<<<(unsigned)cdiv(M, LN_ROWS), 256, 0, V.st>>>(X, M, D, D, B.n2w, B.n2b, 1e-12f, A, D);
        linear(V, B.fc1, A, M, F, nullptr, true);
        linear(V, B.fc2, F, M, Hn, X, false);   // x + fc2(gelu(fc1(...)))
        std::swap(X, Hn);
    }
    // LayerNorm of the CLS rows (vit.py:100-101)
    k_layernorm<<<(unsigned)cdiv(N, LN_ROWS), 256, 0, V.st>>>(X, N, D, (int64_t)VT * D, V.nw, V.nb, 1e-12f, emb, D);
}

// forward in the handle's operand mode; guarded split-fp16: an operand >= 2^14 (or NaN) anywhere
// raises the flag and the whole forward runs again on fp32 MFMA (same contract as MTCNN's ONet)
static void vit_run(Vit& V, const float* x_nhwc8, int64_t N, float* emb) {
    V.cur_x = V.xmode;
    if (V.cur_x) {
        if (!V.d_ovf) VTF_HIP(hipMalloc((void**)&V.d_ovf, 4));
        VTF_HIP(hipMemsetAsync(V.d_ovf, 0, 4, V.st));
    }
    vit_forward(V, x_nhwc8, N, emb);
    if (V.cur_x) {
        int ovf = 0;
        VTF_HIP(hipMemcpyAsync(&ovf, V.d_ovf, 4, hipMemcpyDeviceToHost, V.st));
        VTF_HIP(hipStreamSynchronize(V.st));
        V.cur_x = 0;
        if (ovf) vit_forward(V, x_nhwc8, N, emb);
    }
}

}  // namespace vtf


using namespace vtf;

struct vtf_vit_s {
    Vit v;
};

extern "C" {

int vtf_vit_create(const float* params, int64_t n_params, int dim, int depth, int device, vtf_vit_t* out) {
    return guarded([&] {
        // dim: 64-wide heads, and k_layernorm's float4-per-lane rows (dim % 256 == 0, <= 1024)
        VTF_CHECK(params && out && dim % 256 == 0 && dim <= 256 * LN_MAXV && depth > 0, VTF_E_ARG,
                  "bad argument (dim must be a multiple of 256, at most 1024)");
        DeviceGuard dg(device);
        auto* h = new vtf_vit_s();
        h->v.device = device;
        h->v.D = dim;
        h->v.depth = depth;
        h->v.heads = dim / 64;
        try {
            vit_build(h->v, params, n_params);
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
    });
}

int vtf_vit_destroy(vtf_vit_t h) {
    return guarded_on(h ? h->v.device : -1, [&] { delete h; });
}

int vtf_vit_set_precision(vtf_vit_t h, int mode) {
    return guarded_on(h ? h->v.device : -1, [&] {
        VTF_CHECK(h && (mode == 0 || mode == 2), VTF_E_ARG, "vit precision: 0 (fp32) or 2 (guarded split-fp16)");
        h->v.xmode = mode;
    });
}

int vtf_vit_set_stream(vtf_vit_t h, void* stream) {
    return guarded_on(h ? h->v.device : -1, [&] {
        VTF_CHECK(h, VTF_E_ARG, "null handle");
        h->v.st = (hipStream_t)stream;
    });
}

int vtf_vit_forward(vtf_vit_t h, const float* d_x, int64_t N, float* d_emb) {
    return guarded_on(h ? h->v.device : -1, [&] {
        VTF_CHECK(h && N >= 0, VTF_E_ARG, "bad argument");
        if (N == 0) return;
        VTF_CHECK(d_x && d_emb, VTF_E_ARG, "null argument");
        float* x8 = h->v.ar.get<float>(6, N * 128 * 128 * 8);
        launch_nchw_to_nhwc(d_x, (int)N, 3, 128, 128, 8, x8, false, h->v.st);
        vit_run(h->v, x8, N, d_emb);
        VTF_HIP(hipGetLastError());
    });
}

int vtf_vit_encode_crops(vtf_vit_t h, const uint8_t* d_frames, int n_frames, int H, int W, int64_t frame_stride,
                         int64_t row_stride, const int32_t* crops, int crops_on_device, int64_t N, float* d_emb) {
    return guarded_on(h ? h->v.device : -1, [&] {
        VTF_CHECK(h && N >= 0 && n_frames > 0 && H > 0 && W > 0, VTF_E_ARG, "bad argument");
        if (N == 0) return;
        VTF_CHECK(d_frames && crops && d_emb, VTF_E_ARG, "null argument");
        const int32_t* dc = crops;
        if (!crops_on_device) {
            check_crops_host(crops, N, n_frames, H, W);
            int32_t* d = h->v.ar.get<int32_t>(7, N * 5);
            VTF_HIP(hipMemcpyAsync(d, crops, N * 5 * 4, hipMemcpyHostToDevice, h->v.st));
            dc = d;
        }
        float* x8 = h->v.ar.get<float>(6, N * 128 * 128 * 8);
        // blobFromImages(images, 1/127.5, (128,128), (127.5,)*3, swapRB=True) (vit.py:141)
        launch_blob(d_frames, n_frames, H, W, frame_stride, row_stride, dc, N, 128, 127.5f, (float)(1.0 / 127.5), 1, 8, false,
                    x8, h->v.st);
        vit_run(h->v, x8, N, d_emb);
        VTF_HIP(hipGetLastError());
    });
}

}  // extern "C"

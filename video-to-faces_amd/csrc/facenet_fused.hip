// FaceNet Block17 (src/videotofaces/encoders/facenet.py:36-56) as ONE launch per block in the
// bf16 mode: one workgroup per image (8 x 8 pixels x 896 channels), the whole branch chain kept
// on chip.
//
// The unfused form is four implicit-GEMM launches per block at batch 128 (M = 8192 rows):
// merged 1x1 896 -> 128|128, 1x7 128 -> 128, 7x1 128 -> 128, 1x1 256 -> 896 + residual -- each a
// latency-bound GEMM (MFMA busy 2-3 %), ~74 us per block.  Here the activations
// between the four GEMMs never leave LDS:
//   stage 1  C1[64][256] = X[64][896] W_m^T, BN + ReLU            -> B1 (LDS, bf16)
//   stage 2  C2[64][128] = im2col_1x7(B1[:, 128:256]) W_a^T, BN+ReLU -> B2 (LDS)
//   stage 3  C3[64][128] = im2col_7x1(B2) W_b^T, BN + ReLU          -> B1[:, 128:256] (the concat)
//   stage 4  Y[64][896] = ReLU(0.1 (B1 W_o^T + b_o) + X)            -> HBM, 7 passes of 128 channels
// Weights stream HBM/L2 -> LDS through an LDS-DMA ring (global_load_lds_dwordx4, counted vmcnt,
// one barrier per k-step); the stage-1 input rows ride in the same ring.  Every GEMM runs the
// unfused kernels' k order -- 32-deep v_mfma_f32_16x16x32_bf16 chunks in ascending k from a zero
// accumulator -- and the same epilogue arithmetic (conv_dev.hpp conv_epilogue8), so the block's
// output is bit-identical to the four launches (tests/test_facenet_gpu.py).
//
// LDS images: weight / X rows of 128 B (one 64-deep k-step), 16-B slot s of row r holding source
// slot s ^ ((r >> 1) & 7) (swizzle applied on the DMA source address; conflict-free fragment
// reads, as conv_dma.hip); B1 / B2 rows padded to 528 / 272 B so the 16 rows of a fragment read
// land on 16 distinct bank slots.
#include <algorithm>

#include "common.hpp"
#include "conv.hpp"
#include "conv_dev.hpp"

namespace vtf {

namespace {

constexpr int RB = 128;                 // image row bytes per 64-deep k-step
constexpr int B1S = 256 * 2 + 16;       // B1 row stride (bytes): 256 channels + pad
constexpr int B2S = 128 * 2 + 16;       // B2 row stride
constexpr int S1_X = 64 * RB;           // stage-1 slot: X rows (8 KB) ...
constexpr int S1_SLOT = S1_X + 256 * RB;  // ... + W_m rows (32 KB)
constexpr int S1_R = 3;                 // stage-1 ring slots (2 groups in flight)
constexpr int R_OFF = 0;                // ring base
constexpr int B1_OFF = S1_R * S1_SLOT;  // 120 KB
constexpr int ZERO_OFF = B1_OFF + 64 * B1S;
constexpr int LDS_BYTES = ZERO_OFF + 16;
// stages 2-4 reuse the stage-1 ring region: B2 (stages 2-3) / the stage-4 epilogue image E (fp32
// [64][128 + 4]) at its start, then ONE weight ring for all of stages 2-4 (128 rows x 64 k per
// slot; 56 groups: 14 of W_a, 14 of W_b, 28 of W_o) that keeps streaming across the stage
// boundaries and epilogues
constexpr int S2_SLOT = 128 * RB;       // 16 KB
constexpr int S2_R = 5;                 // 4 groups in flight
constexpr int B2_OFF = 0;
constexpr int E_OFF = 0;
constexpr int E_LD = 132;
constexpr int R2_OFF = 64 * E_LD * 4;   // 33,792
static_assert(64 * B2S <= R2_OFF && R2_OFF + S2_R * S2_SLOT <= B1_OFF, "stage 2-4 LDS plan");
static_assert(LDS_BYTES <= 160 * 1024, "LDS plan");

typedef __attribute__((ext_vector_type(4))) float f4;

struct B17P {
    const __bf16* x;  // [N][64][896]
    __bf16* y;
    const __bf16 *wm, *wa, *wb, *wo;  // [256][896], [128][896], [128][896], [896][256]
    const float *alm, *bem, *ala, *bea, *alb, *beb, *bo;
    float scale;
};

__device__ inline void glds16(const void* g, void* l) {
    __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                     (void __attribute__((address_space(3)))*)l, 16, 0, 0);
}

// this wave's DMA groups up to the one N instructions back have landed and its LDS writes are
// done; after the barrier every wave's are
template <int N>
__device__ inline void wait_vm_barrier() {
    asm volatile("s_waitcnt vmcnt(%0) lgkmcnt(0)\n\ts_barrier" ::"n"(N) : "memory");
}

// DMA rows [0, rows) x 128 B (bytes kb .. kb+127 of each row of a matrix with row pitch `pitch`)
// into a swizzled LDS image: rows / 32 one-KB pieces per wave
template <int ROWS>
__device__ inline void dma_rows(const char* src, int64_t pitch, int64_t kb, char* dst, int wave, int lane) {
    const int sl = (lane & 7) ^ (((lane >> 4) + 4 * (wave & 1)) & 7);
#pragma unroll
    for (int j = 0; j < ROWS / 32; j++) {
        const int r = 32 * j + 8 * wave + (lane >> 3);
        glds16(src + r * pitch + kb + sl * 16, dst + (wave + 4 * j) * 1024);
    }
}

// fragment of a swizzled 128-B-row image: rows 16 i + (lane & 15), k half h (0: k 0..31, 1: 32..63)
__device__ inline bf16x8 frag_sw(const char* img, int i, int h, int lane) {
    const int r = lane & 15, s = (4 * h + (lane >> 4)) ^ (r >> 1);
    return *(const bf16x8*)(img + (16 * i + r) * RB + s * 16);
}

__device__ inline float relu_bf(float v) { return fmaxf(v, 0.f); }

// workgroup barrier for LDS traffic only: __syncthreads() would also wait vmcnt(0), draining the
// weight DMAs in flight
__device__ inline void lds_barrier() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }

// BN + ReLU epilogue of a [64][NC-per-wave] accumulator block into an LDS bf16 image
template <int FM, int FN>
__device__ inline void bn_relu_to_lds(const f4 (&acc)[FM][FN], const float* al, const float* be, int n0, char* dst,
                                      int stride, int lane) {
#pragma unroll
    for (int j = 0; j < FN; j++) {
        const int n = n0 + 16 * j + (lane & 15);
        const float a = al[n], b = be[n];
#pragma unroll
        for (int i = 0; i < FM; i++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int m = 16 * i + 4 * (lane >> 4) + q;
                *(__bf16*)(dst + m * stride + n * 2) = (__bf16)relu_bf(fmaf(acc[i][j][q], a, b));
            }
    }
}

__global__ __launch_bounds__(256, 1) void k_block17(B17P p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int img = blockIdx.x;
    const char* X = (const char*)(p.x + (int64_t)img * 64 * 896);
    char* B1 = smem + B1_OFF;
    char* B2 = smem + B2_OFF;
    const char* ZERO = smem + ZERO_OFF;
    if (tid < 4) ((float*)(smem + ZERO_OFF))[tid] = 0.f;
    // stages 2-4's weight groups (see below)
    auto issue2 = [&](int g) {
        const char* w;
        int64_t pitch, kb;
        if (g < 28) {
            w = (const char*)(g < 14 ? p.wa : p.wb);
            pitch = 896 * 2;
            kb = (int64_t)(g % 14) * RB;
        } else {
            w = (const char*)p.wo + (int64_t)((g - 28) >> 2) * 128 * 256 * 2;
            pitch = 256 * 2;
            kb = (int64_t)((g - 28) & 3) * RB;
        }
        dma_rows<128>(w, pitch, kb, smem + R2_OFF + (g % S2_R) * S2_SLOT, wave, lane);
    };

    // ---------------- stage 1: X[64][896] x W_m^T -> B1 (wave: output channels 64 wave .. +64)
    {
        constexpr int S = 14, G = 2 + 8;  // k-steps; DMA instructions per wave per group
        auto issue = [&](int s) {
            char* slot = smem + R_OFF + (s % S1_R) * S1_SLOT;
            dma_rows<64>(X, 896 * 2, (int64_t)s * RB, slot, wave, lane);
            dma_rows<256>((const char*)p.wm, 896 * 2, (int64_t)s * RB, slot + S1_X, wave, lane);
        };
        f4 acc[4][4];
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j < 4; j++) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
        issue(0);
        issue(1);
        for (int s = 0; s < S; s++) {
            if (s + 1 < S)
                wait_vm_barrier<G>();
            else
                wait_vm_barrier<0>();
            if (s + 2 < S) issue(s + 2);
            const char* slot = smem + R_OFF + (s % S1_R) * S1_SLOT;
            const char* W = slot + S1_X + 64 * wave * RB;
#pragma unroll
            for (int h = 0; h < 2; h++) {
                bf16x8 b[4];
#pragma unroll
                for (int j = 0; j < 4; j++) b[j] = frag_sw(W, j, h, lane);
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const bf16x8 a = frag_sw(slot, i, h, lane);
#pragma unroll
                    for (int j = 0; j < 4; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[j], acc[i][j], 0, 0, 0);
                }
            }
        }
        // stages 2-4's first weight groups go out before the epilogue (the stage-1 ring is free once
        // every wave is past this barrier), so the ring never restarts
        lds_barrier();
        issue2(0);
        issue2(1);
        issue2(2);
        issue2(3);
        bn_relu_to_lds<4, 4>(acc, p.alm, p.bem, 64 * wave, B1, B1S, lane);
    }

    // ---------------- stages 2-4 on one weight ring (wave: output channels 32 wave .. +32)
    //   groups  0..13: 1 x 7 on B1[:, 128:256] -> B2         (k = tap * 128 + channel)
    //   groups 14..27: 7 x 1 on B2 -> B1[:, 128:256]
    //   groups 28..55: pass (g - 28) / 4 of W_o (128 output channels), k-step (g - 28) % 4
    {
        constexpr int NG = 56, G = 4;
        f4 acc[4][2];
        const int r = lane & 15, kq = 8 * (lane >> 4);
        float* E = (float*)(smem + E_OFF);
        char* Y = (char*)(p.y + (int64_t)img * 64 * 896);
        int issued = 4;
        for (int g = 0; g < NG; g++) {
            const int ahead = issued - g - 1;
            if (ahead >= 3)
                wait_vm_barrier<3 * G>();
            else if (ahead == 2)
                wait_vm_barrier<2 * G>();
            else if (ahead == 1)
                wait_vm_barrier<G>();
            else
                wait_vm_barrier<0>();
            if (issued < NG) issue2(issued++);
            const int st = g < 14 ? 0 : (g < 28 ? 1 : 2), ks = st < 2 ? g - 14 * st : (g - 28) & 3;
            if (st < 2 ? ks == 0 : ks == 0) {
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int j = 0; j < 2; j++) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
            }
            const char* W = smem + R2_OFF + (g % S2_R) * S2_SLOT + 32 * wave * RB;
#pragma unroll
            for (int h = 0; h < 2; h++) {
                bf16x8 b[2];
#pragma unroll
                for (int j = 0; j < 2; j++) b[j] = frag_sw(W, j, h, lane);
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const char* src;
                    if (st < 2) {  // 1 x 7 / 7 x 1 implicit GEMM: tap ks / 2, channels 64 (ks & 1) + 32 h
                        const int t = ks >> 1, y = 2 * i + (r >> 3), x = r & 7;
                        const int yy = st == 0 ? y : y + t - 3, xx = st == 0 ? x + t - 3 : x;
                        const bool ok = (unsigned)yy < 8u && (unsigned)xx < 8u;
                        const int c = 64 * (ks & 1) + 32 * h + kq;
                        src = !ok ? ZERO : (st == 0 ? B1 + (yy * 8 + xx) * B1S + (128 + c) * 2 : B2 + (yy * 8 + xx) * B2S + c * 2);
                    } else {
                        src = B1 + (16 * i + r) * B1S + (64 * ks + 32 * h + kq) * 2;
                    }
                    const bf16x8 a = *(const bf16x8*)src;
#pragma unroll
                    for (int j = 0; j < 2; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[j], acc[i][j], 0, 0, 0);
                }
            }
            if (st < 2 && ks == 13) {
                // BN + ReLU into the next operand (read only after the next group's barrier)
                const float* al = st == 0 ? p.ala : p.alb;
                const float* be = st == 0 ? p.bea : p.beb;
                if (st == 0)
                    bn_relu_to_lds<4, 2>(acc, al, be, 32 * wave, B2, B2S, lane);
                else
                    bn_relu_to_lds<4, 2>(acc, al, be, 32 * wave, B1 + 128 * 2, B1S, lane);
            } else if (st == 2 && ks == 3) {
                // pass epilogue through the fp32 image E (B2 is dead by now): 8 consecutive channels
                // per thread (16-B residual loads and output stores), conv_epilogue8's arithmetic;
                // E is rewritten four groups (four barriers) later
                const int pass = (g - 28) >> 2;
#pragma unroll
                for (int i = 0; i < 4; i++)
#pragma unroll
                    for (int j = 0; j < 2; j++)
#pragma unroll
                        for (int q = 0; q < 4; q++)
                            E[(16 * i + 4 * (lane >> 4) + q) * E_LD + 32 * wave + 16 * j + (lane & 15)] = acc[i][j][q];
                lds_barrier();
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    const int e = tid + 256 * u, m = e >> 4, gg = e & 15, c0 = pass * 128 + 8 * gg;
                    const f4 lo = *(const f4*)(E + m * E_LD + 8 * gg), hi = *(const f4*)(E + m * E_LD + 8 * gg + 4);
                    const float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    const bf16x8 rx = *(const bf16x8*)(X + ((int64_t)m * 896 + c0) * 2);
                    bf16x8 o;
#pragma unroll
                    for (int k = 0; k < 8; k++) {
                        float t = v[k] + p.bo[c0 + k];
                        if (p.scale != 1.f) t = t * p.scale;
                        t = t + (float)rx[k];
                        o[k] = (__bf16)fmaxf(t, 0.f);
                    }
                    *(bf16x8*)(Y + ((int64_t)m * 896 + c0) * 2) = o;
                }
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Block35 branches (facenet.py:14-33) in one launch per block: one workgroup per image (17 x 17
// pixels, 289 rows padded to 19 fragments of 16), waves split the rows (fragments w, w+4, ...).
//   stage 1  C1[289][96] = X[289][256] W_m^T (merged heads b0 | b1 | b2), BN + ReLU:
//            b0 -> CAT[:, 0:32] (HBM), b1 / b2 heads -> T[:, 0:64] (LDS)
//   stage 2  3x3 32 -> 32 on T[:, 0:32]   -> CAT[:, 32:64]
//   stage 3  3x3 32 -> 32 on T[:, 32:64]  -> T[:, 0:32] (b2 middle)
//   stage 4  3x3 32 -> 32 on T[:, 0:32]   -> CAT[:, 64:96]
// The block tail (1x1 96 -> 256 + residual) stays one implicit-GEMM launch on CAT.  Operands
// straight from global memory into registers (each wave owns its rows; the weights are small and
// L2-resident), one 32-deep chunk ahead; same k order and epilogue as the unfused launches.
constexpr int T5S = 64 * 2 + 16;  // T row stride (bytes)
constexpr int B35_ROWS = 289, B35_FR = 19;
constexpr int WM5S = 256 * 2 + 16, W35S = 288 * 2 + 16;  // resident weight row strides (conflict-free)
constexpr int B35_WM = 0, B35_W3 = B35_WM + 96 * WM5S, B35_T = B35_W3 + 3 * 32 * W35S;
constexpr int B35_ZERO = B35_T + B35_FR * 16 * T5S;
constexpr int B35_LDS = B35_ZERO + 16;
static_assert(B35_LDS <= 160 * 1024, "Block35 LDS plan");

struct B35P {
    const __bf16* x;  // [N][289][256]
    __bf16* cat;      // [N][289][96]
    const __bf16 *wm, *w1, *w2a, *w2b;  // [96][256], [32][288] x 3
    const float *alm, *bem, *al1, *be1, *al2a, *be2a, *al2b, *be2b;
};

template <int NF>
__device__ inline void b35_store(const f4 (&acc)[5][NF], int nf, int wave, int lane, int n0, const float* al,
                                 const float* be, int oc, char* lds, int lstride, int lcoff, __bf16* g, int gcoff) {
#pragma unroll
    for (int j = 0; j < NF; j++) {
        const int n = n0 + 16 * j + (lane & 15);
        const float a = al[n], b = be[n];
#pragma unroll
        for (int f = 0; f < 5; f++) {
            if (f >= nf) break;
            const int fr = wave + 4 * f;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int m = 16 * fr + 4 * (lane >> 4) + q;
                if (m >= B35_ROWS) continue;
                const __bf16 v = (__bf16)relu_bf(fmaf(acc[f][j][q], a, b));
                const int c = n - oc;  // channel within the destination
                if (g)
                    g[(int64_t)m * 96 + gcoff + c] = v;
                else
                    *(__bf16*)(lds + m * lstride + (lcoff + c) * 2) = v;
            }
        }
    }
}

// Block35 branches: every weight (103 KB) resident in LDS from the start (one burst of loads), so
// the only global reads in the loops are the wave's own input rows (stage 1, three chunks ahead)
__global__ __launch_bounds__(256, 1) void k_block35_br(B35P p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int img = blockIdx.x;
    const int nf = wave < 3 ? 5 : 4;  // fragments w, w + 4, ..., < 19
    char* T = smem + B35_T;
    const char* ZERO = smem + B35_ZERO;
    if (tid < 4) ((float*)(smem + B35_ZERO))[tid] = 0.f;
    const __bf16* X = p.x + (int64_t)img * B35_ROWS * 256;
    __bf16* CAT = p.cat + (int64_t)img * B35_ROWS * 96;
    const int r = lane & 15, kq = 8 * (lane >> 4);
    // weights -> LDS (padded rows)
    for (int e = tid; e < 96 * 32; e += 256) {
        const int n = e >> 5, c = e & 31;
        *(bf16x8*)(smem + B35_WM + n * WM5S + c * 16) = *(const bf16x8*)(p.wm + n * 256 + 8 * c);
    }
    for (int e = tid; e < 3 * 32 * 36; e += 256) {
        const int cv = e / (32 * 36), rem = e - cv * 32 * 36, n = rem / 36, c = rem - n * 36;
        const __bf16* w = cv == 0 ? p.w1 : (cv == 1 ? p.w2a : p.w2b);
        *(bf16x8*)(smem + B35_W3 + (cv * 32 + n) * W35S + c * 16) = *(const bf16x8*)(w + n * 288 + 8 * c);
    }

    // ---- stage 1 (K = 256: 8 chunks of 32; N = 96: 6 fragments); input rows 3 chunks ahead
    {
        f4 acc[5][6];
#pragma unroll
        for (int f = 0; f < 5; f++)
#pragma unroll
            for (int j = 0; j < 6; j++) acc[f][j] = f4{0.f, 0.f, 0.f, 0.f};
        const bf16x8* arow[5];
#pragma unroll
        for (int f = 0; f < 5; f++) {
            const int m = min(16 * (wave + 4 * f) + r, B35_ROWS - 1);  // padding rows: any finite row
            arow[f] = (const bf16x8*)(X + (int64_t)m * 256 + kq);
        }
        bf16x8 a[4][5];
#pragma unroll
        for (int c = 0; c < 3; c++)
#pragma unroll
            for (int f = 0; f < 5; f++) a[c][f] = arow[f][4 * c];
        __syncthreads();  // resident weights stored
#pragma unroll
        for (int c = 0; c < 8; c++) {
            if (c + 3 < 8)
#pragma unroll
                for (int f = 0; f < 5; f++) a[(c + 3) & 3][f] = arow[f][4 * (c + 3)];
            bf16x8 b[6];
#pragma unroll
            for (int j = 0; j < 6; j++) b[j] = *(const bf16x8*)(smem + B35_WM + (16 * j + r) * WM5S + (32 * c + kq) * 2);
#pragma unroll
            for (int f = 0; f < 5; f++)
                if (f < nf)
#pragma unroll
                    for (int j = 0; j < 6; j++)
                        acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[c & 3][f], b[j], acc[f][j], 0, 0, 0);
        }
        // b0 (channels 0..31) -> CAT[:, 0:32]; heads (32..95) -> T[:, 0:64]
        f4 a0[5][2], a1[5][4];
#pragma unroll
        for (int f = 0; f < 5; f++) {
            a0[f][0] = acc[f][0];
            a0[f][1] = acc[f][1];
#pragma unroll
            for (int j = 0; j < 4; j++) a1[f][j] = acc[f][2 + j];
        }
        b35_store<2>(a0, nf, wave, lane, 0, p.alm, p.bem, 0, nullptr, 0, 0, CAT, 0);
        b35_store<4>(a1, nf, wave, lane, 32, p.alm, p.bem, 32, T, T5S, 0, nullptr, 0);
    }
    __syncthreads();

    // ---- 3x3 32 -> 32, pad 1, on T[:, icoff : icoff + 32] (K = 9 taps x 32: one chunk per tap)
    int py[5], px[5];
#pragma unroll
    for (int f = 0; f < 5; f++) {
        const int m = 16 * (wave + 4 * f) + r;
        py[f] = m < B35_ROWS ? m / 17 : -100;
        px[f] = m < B35_ROWS ? m - 17 * (m / 17) : 0;
    }
    auto conv3 = [&](int cv, const float* al, const float* be, int icoff, char* lds_out, int lcoff, int gcoff) {
        f4 acc[5][2];
#pragma unroll
        for (int f = 0; f < 5; f++)
#pragma unroll
            for (int j = 0; j < 2; j++) acc[f][j] = f4{0.f, 0.f, 0.f, 0.f};
        const char* W = smem + B35_W3 + cv * 32 * W35S;
#pragma unroll
        for (int t = 0; t < 9; t++) {
            bf16x8 b[2];
#pragma unroll
            for (int j = 0; j < 2; j++) b[j] = *(const bf16x8*)(W + (16 * j + r) * W35S + (32 * t + kq) * 2);
            const int dy = t / 3 - 1, dx = t % 3 - 1;
#pragma unroll
            for (int f = 0; f < 5; f++) {
                if (f >= nf) break;
                const int yy = py[f] + dy, xx = px[f] + dx;
                const bool ok = (unsigned)yy < 17u && (unsigned)xx < 17u;
                const char* src = ok ? T + (yy * 17 + xx) * T5S + (icoff + kq) * 2 : ZERO;
                const bf16x8 a = *(const bf16x8*)src;
#pragma unroll
                for (int j = 0; j < 2; j++) acc[f][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[j], acc[f][j], 0, 0, 0);
            }
        }
        __syncthreads();  // every wave is done reading T before a stage writes it
        b35_store<2>(acc, nf, wave, lane, 0, al, be, 0, lds_out, T5S, lcoff, lds_out ? nullptr : CAT, gcoff);
        __syncthreads();
    };
    conv3(0, p.al1, p.be1, 0, nullptr, 0, 32);    // b1: T[:, 0:32] -> CAT[:, 32:64]
    conv3(1, p.al2a, p.be2a, 32, T, 0, 0);       // b2 middle: T[:, 32:64] -> T[:, 0:32]
    conv3(2, p.al2b, p.be2b, 0, nullptr, 0, 64);  // b2 tail: T[:, 0:32] -> CAT[:, 64:96]
}

// ---------------------------------------------------------------------------------------------
// FaceNet stem 3x3 stride-1 convs with few input channels (conv2d_2a 32 -> 32, conv2d_2b 32 -> 64,
// facenet.py:127-128) as "patch" convs: a tile of 8 x 16 output pixels reads its (8+2) x (16+2)
// input patch once into LDS and all nine taps from there.  The implicit-GEMM launches gathered
// every tap from L2 (9x the input bytes: ~0.5 GB per enc-batch for conv2d_2b, L2-bound).
// Persistent workgroups (weights staged in LDS once), the next tile's patch loaded into registers
// during the current tile's MFMAs.  k order (tap-major, 32 channels per chunk) and the BN + ReLU
// epilogue are the unfused kernels', so the output is bit-identical.
constexpr int CP_TH = 8, CP_TW = 16, CP_PH = CP_TH + 2, CP_PW = CP_TW + 2, CP_CIN = 32;
constexpr int CP_PS = CP_CIN * 2 + 16;     // patch pixel stride (bytes): 16 consecutive pixels -> 16 bank slots
constexpr int CP_WS = 9 * CP_CIN * 2 + 16;  // weight row stride (bytes)
constexpr int CP_PIECES = CP_PH * CP_PW * CP_CIN * 2 / 16;  // 16-B patch pieces (720)
constexpr int CP_PPT = (CP_PIECES + 255) / 256;             // per thread

struct CPatchP {
    const __bf16* in;  // [N][H][W][32]
    __bf16* out;       // [N][OH][OW][COUT]
    const __bf16* w;   // [COUT][9 * 32]
    const float *al, *be;
    int N, H, W, OH, OW, pad, tiles_x, tiles_y, tiles;
};

template <int COUT>
__global__ __launch_bounds__(256, 2) void k_conv_patch(CPatchP p) {
    constexpr int FN = COUT / 16;
    extern __shared__ __attribute__((aligned(16))) char smem[];
    char* Wl = smem;                              // [COUT][CP_WS]
    char* P = smem + COUT * CP_WS;                // patch [CP_PH * CP_PW][CP_PS]
    char* E = P + CP_PH * CP_PW * CP_PS;          // output staging [128][COUT] bf16
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // weights once per workgroup
    for (int e = tid; e < COUT * 9 * CP_CIN / 8; e += 256) {
        const int n = e / (9 * CP_CIN / 8), c = e - n * (9 * CP_CIN / 8);
        *(bf16x8*)(Wl + n * CP_WS + c * 16) = *(const bf16x8*)(p.w + (int64_t)n * 9 * CP_CIN + 8 * c);
    }
    float al[FN], be[FN];
#pragma unroll
    for (int j = 0; j < FN; j++) {
        al[j] = p.al[16 * j + (lane & 15)];
        be[j] = p.be[16 * j + (lane & 15)];
    }
    auto tile_geo = [&](int t, int& n, int& oy0, int& ox0) {
        const int per = p.tiles_x * p.tiles_y;
        n = t / per;
        const int r = t - n * per, ty = r / p.tiles_x;
        oy0 = ty * CP_TH;
        ox0 = (r - ty * p.tiles_x) * CP_TW;
    };
    bf16x8 pr[CP_PPT];
    auto load_patch = [&](int t) {
        int n, oy0, ox0;
        tile_geo(t, n, oy0, ox0);
#pragma unroll
        for (int u = 0; u < CP_PPT; u++) {
            const int e = tid + 256 * u;
            bf16x8 v = {};
            if (e < CP_PIECES) {
                const int pix = e >> 2, c = e & 3;  // 4 pieces of 8 channels per pixel
                const int py = pix / CP_PW, px = pix - py * CP_PW;
                const int iy = oy0 - p.pad + py, ix = ox0 - p.pad + px;
                if ((unsigned)iy < (unsigned)p.H && (unsigned)ix < (unsigned)p.W)
                    v = *(const bf16x8*)(p.in + (((int64_t)n * p.H + iy) * p.W + ix) * CP_CIN + 8 * c);
            }
            pr[u] = v;
        }
    };
    auto store_patch = [&]() {
#pragma unroll
        for (int u = 0; u < CP_PPT; u++) {
            const int e = tid + 256 * u;
            if (e < CP_PIECES) *(bf16x8*)(P + (e >> 2) * CP_PS + (e & 3) * 16) = pr[u];
        }
    };
    int t = blockIdx.x;
    if (t < p.tiles) load_patch(t);
    // the lane's two A rows (fragments 2 wave, 2 wave + 1): tile pixel (ty, tx)
    const int r = lane & 15, kq = 8 * (lane >> 4);
    for (; t < p.tiles; t += gridDim.x) {
        __syncthreads();  // the previous tile's patch and staging reads are done (weights on the first pass)
        store_patch();
        __syncthreads();
        if (t + gridDim.x < p.tiles) load_patch(t + gridDim.x);
        f4 acc[2][FN];
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int j = 0; j < FN; j++) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int tap = 0; tap < 9; tap++) {
            const int dy = tap / 3, dx = tap % 3;
            bf16x8 b[FN];
#pragma unroll
            for (int j = 0; j < FN; j++) b[j] = *(const bf16x8*)(Wl + (16 * j + r) * CP_WS + (tap * CP_CIN + kq) * 2);
#pragma unroll
            for (int i = 0; i < 2; i++) {
                const int m = 16 * (2 * wave + i) + r, ty = m >> 4, tx = m & 15;
                const bf16x8 a = *(const bf16x8*)(P + ((ty + dy) * CP_PW + tx + dx) * CP_PS + kq * 2);
#pragma unroll
                for (int j = 0; j < FN; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[j], acc[i][j], 0, 0, 0);
            }
        }
        // BN + ReLU -> bf16 staging [128][COUT] -> 16-B stores of the in-bounds pixels
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int j = 0; j < FN; j++)
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int m = 16 * (2 * wave + i) + 4 * (lane >> 4) + q;
                    *(__bf16*)(E + (m * COUT + 16 * j + (lane & 15)) * 2) = (__bf16)relu_bf(fmaf(acc[i][j][q], al[j], be[j]));
                }
        __syncthreads();
        int n, oy0, ox0;
        tile_geo(t, n, oy0, ox0);
        for (int e = tid; e < 128 * COUT / 8; e += 256) {
            const int m = e / (COUT / 8), c = e - m * (COUT / 8);
            const int oy = oy0 + (m >> 4), ox = ox0 + (m & 15);
            if (oy < p.OH && ox < p.OW)
                *(bf16x8*)(p.out + (((int64_t)n * p.OH + oy) * p.OW + ox) * COUT + 8 * c) = *(const bf16x8*)(E + (m * COUT + 8 * c) * 2);
        }
    }
}

}  // namespace

// one Block17 (bf16 NHWC [N, 8, 8, 896] -> same): weights as FaceNet's layer table holds them
void launch_block17_fused(const void* x, void* y, int N, const void* wm, const float* alm, const float* bem,
                          const void* wa, const float* ala, const float* bea, const void* wb, const float* alb,
                          const float* beb, const void* wo, const float* bo, float scale, hipStream_t st) {
    if (N <= 0) return;
    B17P p;
    p.x = (const __bf16*)x;
    p.y = (__bf16*)y;
    p.wm = (const __bf16*)wm;
    p.wa = (const __bf16*)wa;
    p.wb = (const __bf16*)wb;
    p.wo = (const __bf16*)wo;
    p.alm = alm;
    p.bem = bem;
    p.ala = ala;
    p.bea = bea;
    p.alb = alb;
    p.beb = beb;
    p.bo = bo;
    p.scale = scale;
    static bool attr = [] {
        VTF_HIP(hipFuncSetAttribute((const void*)k_block17, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES));
        return true;
    }();
    (void)attr;
    k_block17<<<N, 256, LDS_BYTES, st>>>(p);
    VTF_HIP(hipGetLastError());
}

}  // namespace vtf

namespace vtf {

// Block35 branches (bf16 NHWC [N, 17, 17, 256] -> CAT [N, 17, 17, 96])
void launch_block35_branches(const void* x, void* cat, int N, const void* wm, const float* alm, const float* bem,
                             const void* w1, const float* al1, const float* be1, const void* w2a, const float* al2a,
                             const float* be2a, const void* w2b, const float* al2b, const float* be2b,
                             hipStream_t st) {
    if (N <= 0) return;
    B35P p;
    p.x = (const __bf16*)x;
    p.cat = (__bf16*)cat;
    p.wm = (const __bf16*)wm;
    p.w1 = (const __bf16*)w1;
    p.w2a = (const __bf16*)w2a;
    p.w2b = (const __bf16*)w2b;
    p.alm = alm;
    p.bem = bem;
    p.al1 = al1;
    p.be1 = be1;
    p.al2a = al2a;
    p.be2a = be2a;
    p.al2b = al2b;
    p.be2b = be2b;
    static bool attr = [] {
        VTF_HIP(hipFuncSetAttribute((const void*)k_block35_br, hipFuncAttributeMaxDynamicSharedMemorySize, B35_LDS));
        return true;
    }();
    (void)attr;
    k_block35_br<<<N, 256, B35_LDS, st>>>(p);
    VTF_HIP(hipGetLastError());
}

}  // namespace vtf

namespace vtf {

static int cus() {
    static int n = [] {
        int dev = 0, c = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev);
        return c;
    }();
    return n;
}

// FaceNet stem patch conv (3x3, stride 1, 32 input channels, bf16; cout 32 or 64); false = not this shape
bool launch_conv_patch(const ConvParams& q, hipStream_t st) {
    if (q.Cin != CP_CIN || q.KH != 3 || q.KW != 3 || q.sh != 1 || q.sw != 1 || q.ph != q.pw || q.ph > 1 ||
        (q.Cout != 32 && q.Cout != 64) || q.in_cstride || q.out_cstride != q.Cout || q.out_coff || q.res || q.bias ||
        !q.alpha || !q.relu || q.n_split)
        return false;
    CPatchP p;
    p.in = (const __bf16*)q.in;
    p.out = (__bf16*)q.out;
    p.w = (const __bf16*)q.w;
    p.al = q.alpha;
    p.be = q.beta;
    p.N = q.N;
    p.H = q.H;
    p.W = q.W;
    p.OH = q.OH;
    p.OW = q.OW;
    p.pad = q.ph;
    p.tiles_x = (q.OW + CP_TW - 1) / CP_TW;
    p.tiles_y = (q.OH + CP_TH - 1) / CP_TH;
    p.tiles = q.N * p.tiles_x * p.tiles_y;
    if (p.tiles <= 0) return true;
    const int grid = std::min(p.tiles, 2 * cus());
    const size_t lds = (size_t)q.Cout * CP_WS + CP_PH * CP_PW * CP_PS + 128 * q.Cout * 2;
    static bool attr = [] {
        for (const void* f : {(const void*)k_conv_patch<32>, (const void*)k_conv_patch<64>})
            VTF_HIP(hipFuncSetAttribute(f, hipFuncAttributeMaxDynamicSharedMemorySize,
                                        64 * CP_WS + CP_PH * CP_PW * CP_PS + 128 * 64 * 2));
        return true;
    }();
    (void)attr;
    if (q.Cout == 32)
        k_conv_patch<32><<<grid, 256, lds, st>>>(p);
    else
        k_conv_patch<64><<<grid, 256, lds, st>>>(p);
    VTF_HIP(hipGetLastError());
    return true;
}

}  // namespace vtf

// FaceNet bf16 blocks as single launches (src/videotofaces/encoders/facenet.py:14-56, 126-128).
//
// Block17 as ONE launch per block: one workgroup per image (8 x 8 pixels x 896 channels), the
// whole branch chain kept on chip.
//
// The unfused form is four implicit-GEMM launches per block at batch 128 (M = 8192 rows):
// merged 1x1 896 -> 128|128, 1x7 128 -> 128, 7x1 128 -> 128, 1x1 256 -> 896 + residual -- each a
// latency-bound GEMM (MFMA busy 2-3 %), ~74 us per block.  Here the activations
// between the four GEMMs never leave LDS:
//   stage 1  C1[64][256] = X[64][896] W_m^T, BN + ReLU            -> B1 (LDS, bf16)
//   stage 2  C2[64][128] = im2col_1x7(B1[:, 128:256]) W_a^T, BN+ReLU -> B2 (LDS)
//   stage 3  C3[64][128] = im2col_7x1(B2) W_b^T, BN + ReLU          -> B1[:, 128:256] (the concat)
//   stage 4  Y[64][896] = ReLU(0.1 (B1 W_o^T + b_o) + X)            -> HBM, 7 passes of 128 channels
// Every GEMM runs the unfused kernels' k order -- 32-deep v_mfma_f32_16x16x32_bf16 chunks in
// ascending k from a zero accumulator -- and the same epilogue arithmetic (conv_dev.hpp
// conv_epilogue8); the unfused launches split K on small grids (VTF_NO_SPLITK=1 turns that off: then
// the two paths are bit-identical), so by default the two paths agree to bf16
// rounding (identical at small batches; tests/test_facenet_gpu.py).  LDS images are padded (row
// strides 16 B past a multiple of 256 B) so the 16 rows of a fragment read land on 16 distinct
// bank slots.
//
// What bounds it (measured, VTF_B17_CLK stage clocks): every workgroup streams the block's 1.38 MB
// of weights from L2, at ~12 B/cycle per CU -- the same per-CU L2 rate the unfused 64 x 64 GEMM
// tiles run at.  An LDS-DMA weight ring (57 us: ~150 cycles of issue per 1-KB piece), register
// rings 4 and 8 chunks deep, an L2 warm-up and free scheduling all measured within 3 % of each
// other: 57 us per block against 74 us for the four launches.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "blob.hpp"
#include "common.hpp"
#include "conv.hpp"
#include "conv_dev.hpp"

namespace vtf {

namespace {

constexpr int B1S = 256 * 2 + 16;       // B1 row stride (bytes): 256 channels + pad
constexpr int B2S = 128 * 2 + 16;       // B2 row stride
constexpr int E_LD = 132;               // stage-4 fp32 epilogue image row stride (floats)

typedef __attribute__((ext_vector_type(4))) float f4;

struct B17P {
    const __bf16* x;  // [N][64][896]
    __bf16* y;
    const __bf16 *wm, *wa, *wb, *wo;  // [256][896], [128][896], [128][896], [896][256]
    const float *alm, *bem, *ala, *bea, *alb, *beb, *bo;
    float scale;
    // row stride (elements) of wm / wa / wb: 896, or padded (facenet_runtime: a stride that is a
    // multiple of 128 B puts the 16 rows one load instruction reads -- 64 B each -- at the same
    // offset in their cache lines, and the block ran ~25 % slower, scripts/r06_b17ws.py)
    int ws;
    int wos;  // row stride (elements) of wo: 256, or padded likewise
    unsigned long long* clk;  // debug (VTF_B17_CLK): thread 0's shader clock at the stage ends, [N][5]
};

__device__ inline float relu_bf(float v) { return fmaxf(v, 0.f); }

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

// Weight fragments stream straight from L2 into registers (each wave loads only its own output
// channels' rows: no redundancy, no LDS staging); chunk c + R - 1's loads are issued while chunk c
// computes (R = 8 chunks of 32 k).
constexpr int X_S = 896 * 2 + 16;          // resident input image row stride (bytes)
constexpr int K17_X = 0;                    // X image [64][X_S] (stage 1), then B2 / E (stages 2-4)
constexpr int K17_B1 = 64 * X_S;            // 115,712
constexpr int K17_ZERO = K17_B1 + 64 * B1S;
constexpr int K17_LDS = K17_ZERO + 16;
constexpr int K17_E = 64 * B2S;             // E after B2 (stage 4 only; B2 is dead by then anyway)
static_assert(K17_E + 64 * E_LD * 4 <= K17_B1 && K17_LDS <= 160 * 1024, "Block17 LDS plan");

// chunk loop with a register ring of R chunks: load(c, slot) issues chunk c's fragments into ring
// slot `slot` (compile-time), comp(c, slot) consumes them
template <int NC, int R, class L, class C>
__device__ inline void reg_ring(L load, C comp) {
#pragma unroll
    for (int u = 0; u < R - 1 && u < NC; u++) load(u, u % R);
    __builtin_amdgcn_sched_barrier(0);
    // fully unrolled (slots are compile-time): hipcc's waitcnt insertion is exact on straight-line
    // code, conservative across a loop back-edge; the sched_barriers keep the loads where they
    // are (the machine scheduler otherwise sinks them next to their use: vmcnt(1) waits, no overlap)
#pragma unroll
    for (int c = 0; c < NC; c++) {
        if (c + R - 1 < NC) load(c + R - 1, (c + R - 1) % R);
        __builtin_amdgcn_sched_barrier(0);
        comp(c, c % R);
    }
}

// HEAD: stages 1-3 only, the concat B1 [64][256] to p.y ([N][64][256]); stage 4 then runs as one
// GEMM launch over the whole batch (facenet_runtime: all CUs share Wo instead of every image's
// workgroup streaming it)
template <bool HEAD>
__global__ __launch_bounds__(256, 1) void k_block17(B17P p) {
    extern __shared__ __attribute__((aligned(16))) char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int img = blockIdx.x;
    const char* X = (const char*)(p.x + (int64_t)img * 64 * 896);
    char* XL = smem + K17_X;
    char* B1 = smem + K17_B1;
    char* B2 = smem + K17_X;
    const char* ZERO = smem + K17_ZERO;
    const int r = lane & 15, kq = 8 * (lane >> 4);
    auto stamp = [&](int k) {
        if (p.clk && tid == 0) p.clk[img * 5 + k] = clock64();
    };
    stamp(0);
    if (tid < 4) ((float*)(smem + K17_ZERO))[tid] = 0.f;
    // L2 warm-up: the 128 workgroups read the same weights in lockstep, so every first touch would
    // wait on one HBM miss per XCD; one dword per 128-B line of a 1/16 slice of the block's
    // weights (workgroups go to the 8 XCDs round-robin: the 16 of one XCD cover all of them),
    // consumed (kept live) only after stage 1
    uint32_t wv[4];
    {
        const int LM = 256 * p.ws * 2 / 128, LA = 128 * p.ws * 2 / 128, LO = 896 * p.wos * 2 / 128;
        const int LW = LM + 2 * LA + LO, SL = (LW + 15) / 16;  // (SL <= 4 * 256: the host bounds the strides)
        const int j = (img >> 3) & 15;
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const int l = min(j * SL + tid + 256 * u, LW - 1);
            const char* a = l < LM ? (const char*)p.wm + l * 128
                          : l < LM + LA ? (const char*)p.wa + (l - LM) * 128
                          : l < LM + 2 * LA ? (const char*)p.wb + (l - LM - LA) * 128
                          : (const char*)p.wo + (l - LM - 2 * LA) * 128;
            wv[u] = *(const uint32_t*)a;
        }
    }
    // ---- the input image -> LDS, one burst (7168 16-B pieces, 28 per thread)
    {
        constexpr int NP = 64 * 112 / 256;
        bf16x8 v[NP];
#pragma unroll
        for (int u = 0; u < NP; u++) {
            const int e = tid + 256 * u;
            v[u] = *(const bf16x8*)(X + (e / 112) * 1792 + (e % 112) * 16);
        }
#pragma unroll
        for (int u = 0; u < NP; u++) {
            const int e = tid + 256 * u;
            *(bf16x8*)(XL + (e / 112) * X_S + (e % 112) * 16) = v[u];
        }
    }
    __syncthreads();

    // ---- stage 1: X[64][896] x W_m^T -> B1 (wave: output channels 64 wave .. +64; 28 chunks of 32)
    {
        f4 acc[4][4];
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j < 4; j++) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
        const int ws = p.ws;
        const __bf16* wrow = p.wm + (int64_t)(64 * wave + r) * ws + kq;
        bf16x8 b[8][4];
        reg_ring<28, 8>(
            [&](int c, int sl) {
#pragma unroll
                for (int j = 0; j < 4; j++) b[sl][j] = *(const bf16x8*)(wrow + j * 16 * ws + 32 * c);
            },
            [&](int c, int sl) {
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const bf16x8 a = *(const bf16x8*)(XL + (16 * i + r) * X_S + (32 * c + kq) * 2);
#pragma unroll
                    for (int j = 0; j < 4; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[sl][j], acc[i][j], 0, 0, 0);
                }
            });
        bn_relu_to_lds<4, 4>(acc, p.alm, p.bem, 64 * wave, B1, B1S, lane);
        asm volatile("" ::"v"(wv[0] | wv[1] | wv[2] | wv[3]));
    }
    __syncthreads();  // B1 complete; the X image is dead (B2 / E take its place)
    stamp(1);

    // ---- stages 2 and 3: 1 x 7 / 7 x 1, 128 -> 128 (wave: channels 32 wave .. +32; k = tap * 128 + c)
    auto conv7 = [&](const __bf16* w, bool along_w, const char* in, int in_stride, int in_coff, const float* al,
                     const float* be, char* out, int out_stride) {
        f4 acc[4][2];
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j < 2; j++) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
        const int ws = p.ws;
        const __bf16* wrow = w + (int64_t)(32 * wave + r) * ws + kq;
        bf16x8 b[8][2];
        reg_ring<28, 8>(
            [&](int c, int sl) {
#pragma unroll
                for (int j = 0; j < 2; j++) b[sl][j] = *(const bf16x8*)(wrow + j * 16 * ws + 32 * c);
            },
            [&](int c, int sl) {
                const int t = c >> 2, ch = in_coff + 32 * (c & 3) + kq;
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int y = 2 * i + (r >> 3), x = r & 7;
                    const int yy = along_w ? y : y + t - 3, xx = along_w ? x + t - 3 : x;
                    const bool ok = (unsigned)yy < 8u && (unsigned)xx < 8u;
                    const bf16x8 a = *(const bf16x8*)(ok ? in + (yy * 8 + xx) * in_stride + ch * 2 : ZERO);
#pragma unroll
                    for (int j = 0; j < 2; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[sl][j], acc[i][j], 0, 0, 0);
                }
            });
        bn_relu_to_lds<4, 2>(acc, al, be, 32 * wave, out, out_stride, lane);
        __syncthreads();
    };
    conv7(p.wa, true, B1, B1S, 128, p.ala, p.bea, B2, B2S);
    stamp(2);
    conv7(p.wb, false, B2, B2S, 0, p.alb, p.beb, B1 + 128 * 2, B1S);
    stamp(3);

    if (HEAD) {  // the concat to HBM: 64 rows x 512 B, 16-B pieces
        char* Y = (char*)(p.y + (int64_t)img * 64 * 256);
#pragma unroll
        for (int u = 0; u < 8; u++) {
            const int e = tid + 256 * u;
            *(bf16x8*)(Y + (e >> 5) * 512 + (e & 31) * 16) = *(const bf16x8*)(B1 + (e >> 5) * B1S + (e & 31) * 16);
        }
        stamp(4);
        return;
    }
    // ---- stage 4: B1[64][256] x W_o^T + b_o, x scale, + X, ReLU -> Y; 7 passes of 128 channels
    //      (8 chunks each); two register sets: pass q + 1's weights load during pass q's MFMAs and
    //      epilogue
    {
        float* E = (float*)(smem + K17_E);
        char* Y = (char*)(p.y + (int64_t)img * 64 * 896);
        bf16x8 bA[8][2], bB[8][2];
        auto loadp = [&](int pass, bf16x8(&b)[8][2]) {
#pragma unroll
            for (int cc = 0; cc < 8; cc++)
#pragma unroll
                for (int j = 0; j < 2; j++)
                    b[cc][j] = *(const bf16x8*)(p.wo + (int64_t)(pass * 128 + 32 * wave + 16 * j + r) * p.wos + 32 * cc + kq);
        };
        auto runp = [&](int pass, const bf16x8(&b)[8][2]) {
            bf16x8 rx[4];  // this pass's residual rows (used by its epilogue)
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int e = tid + 256 * u;
                rx[u] = *(const bf16x8*)(X + ((int64_t)(e >> 4) * 896 + pass * 128 + 8 * (e & 15)) * 2);
            }
            f4 acc[4][2];
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < 2; j++) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int cc = 0; cc < 8; cc++)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const bf16x8 a = *(const bf16x8*)(B1 + (16 * i + r) * B1S + (32 * cc + kq) * 2);
#pragma unroll
                    for (int j = 0; j < 2; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, b[cc][j], acc[i][j], 0, 0, 0);
                }
            // 8 consecutive channels per thread (16-B residual loads and output stores),
            // conv_epilogue8's arithmetic
#pragma unroll
            for (int i = 0; i < 4; i++)
#pragma unroll
                for (int j = 0; j < 2; j++)
#pragma unroll
                    for (int q = 0; q < 4; q++)
                        E[(16 * i + 4 * (lane >> 4) + q) * E_LD + 32 * wave + 16 * j + (lane & 15)] = acc[i][j][q];
            __syncthreads();
#pragma unroll
            for (int u = 0; u < 4; u++) {
                const int e = tid + 256 * u, m = e >> 4, gg = e & 15, c0 = pass * 128 + 8 * gg;
                const f4 lo = *(const f4*)(E + m * E_LD + 8 * gg), hi = *(const f4*)(E + m * E_LD + 8 * gg + 4);
                const float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                bf16x8 o;
#pragma unroll
                for (int k = 0; k < 8; k++) {
                    float t = v[k] + p.bo[c0 + k];
                    if (p.scale != 1.f) t = t * p.scale;
                    t = t + (float)rx[u][k];
                    o[k] = (__bf16)fmaxf(t, 0.f);
                }
                *(bf16x8*)(Y + ((int64_t)m * 896 + c0) * 2) = o;
            }
            __syncthreads();  // E is rewritten by the next pass
        };
        loadp(0, bA);
        for (int q = 0; q < 7; q += 2) {
            if (q + 1 < 7) loadp(q + 1, bB);
            __builtin_amdgcn_sched_barrier(0);
            runp(q, bA);
            if (q + 1 < 7) {
                if (q + 2 < 7) loadp(q + 2, bA);
                __builtin_amdgcn_sched_barrier(0);
                runp(q + 1, bB);
            }
        }
    }
    stamp(4);
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
    // weights -> LDS (padded rows): every load of the burst issued before the first store (a
    // load-store loop would pay one global round trip per iteration)
    {
        constexpr int NWM = 96 * 32, NW3 = 3 * 32 * 36, NP = (NWM + NW3 + 255) / 256;  // 16-B pieces
        bf16x8 v[NP];
#pragma unroll
        for (int u = 0; u < NP; u++) {
            const int e = tid + 256 * u;
            if (e < NWM) {
                v[u] = *(const bf16x8*)(p.wm + (e >> 5) * 256 + 8 * (e & 31));
            } else if (e < NWM + NW3) {
                const int e3 = e - NWM, cv = e3 / (32 * 36), rem = e3 - cv * 32 * 36, n = rem / 36, c = rem - n * 36;
                const __bf16* w = cv == 0 ? p.w1 : (cv == 1 ? p.w2a : p.w2b);
                v[u] = *(const bf16x8*)(w + n * 288 + 8 * c);
            }
        }
#pragma unroll
        for (int u = 0; u < NP; u++) {
            const int e = tid + 256 * u;
            if (e < NWM) {
                *(bf16x8*)(smem + B35_WM + (e >> 5) * WM5S + (e & 31) * 16) = v[u];
            } else if (e < NWM + NW3) {
                const int e3 = e - NWM, cv = e3 / (32 * 36), rem = e3 - cv * 32 * 36, n = rem / 36, c = rem - n * 36;
                *(bf16x8*)(smem + B35_W3 + (cv * 32 + n) * W35S + c * 16) = v[u];
            }
        }
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

// ---------------------------------------------------------------------------------------------
// Block8 branch 1 middle (facenet.py:64-68): the 1x3 then the 3x1 conv (192 -> 192, BN + ReLU
// each) on the 3x3 maps as ONE launch for G = 7 images per workgroup (63 pixel rows = 4 MFMA row
// fragments): the branch head's output T1 is staged in LDS, the 1x3 conv's output stays in LDS
// and the 3x1 conv writes CAT[:, 192:384].  Each output's MFMA chain is the unfused launches'
// (k_conv_dma MODE 0 without split-K: nine 64-deep k-steps of (tap, 64-channel block), two
// v_mfma_f32_16x16x32_bf16 per step, the same lane -> k map; taps in the zero padding run with
// zero A), and the epilogue is its fmaf(acc, alpha, beta) + ReLU: bit-identical to the two launches
// (and their split-K tails) it replaces.  Waves own 3 of the 12 output-channel fragments and read
// their weight fragments straight from L2.
constexpr int B8_C = 192, B8_RS = B8_C * 2 + 16;  // LDS row: 384 B + 16 pad

struct B8P {
    const __bf16* t1;   // [N][9][192]
    __bf16* cat;        // [N][9][384]
    const __bf16 *wa, *wb;  // [192][3 * 192]: 1x3 (k = kx * 192 + ci), 3x1 (k = ky * 192 + ci)
    const float *ala, *bea, *alb, *beb;
    int N;
    int ws;  // weight row stride (elements): 576, or padded (see B17P::ws)
};

template <int B8_G>
__global__ __launch_bounds__(256) void k_block8_mid(B8P p) {
    constexpr int B8_PX = 9 * B8_G, NF = (B8_PX + 15) / 16, NR = 16 * NF;
    __shared__ __attribute__((aligned(16))) char X[NR * B8_RS];   // T1 rows (padding rows: zeros)
    __shared__ __attribute__((aligned(16))) char Y[NR * B8_RS];   // 1x3 output rows
    __shared__ __attribute__((aligned(16))) char Z[16];           // zero fragment source
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n0 = blockIdx.x * B8_G, ng = min(B8_G, p.N - n0);
    for (int e = tid; e < NR * (B8_C / 8); e += 256) {
        const int r = e / (B8_C / 8), c = e - r * (B8_C / 8);
        bf16x8 v = {};
        if (r < 9 * ng) v = *(const bf16x8*)(p.t1 + ((int64_t)n0 * 9 + r) * B8_C + 8 * c);
        *(bf16x8*)(X + r * B8_RS + 16 * c) = v;
    }
    if (tid == 0) *(uint4*)Z = make_uint4(0u, 0u, 0u, 0u);
    __syncthreads();
    const int r16 = lane & 15, g = lane >> 4;
    // the lane's A rows: pixel 16 i + r16 (image (.) / 9, y, x) of fragment i
    int py[NF], px[NF];
#pragma unroll
    for (int i = 0; i < NF; i++) {
        const int pix = 16 * i + r16, q = pix % 9;
        py[i] = pix < B8_PX ? q / 3 : -100;  // the padding row reads zeros for every tap
        px[i] = q % 3;
    }
    auto conv = [&](const char* src, const __bf16* w, const float* al, const float* be, bool vertical, int stage) {
        f4 acc[NF][3];
#pragma unroll
        for (int i = 0; i < NF; i++)
#pragma unroll
            for (int j = 0; j < 3; j++) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
        const int nb = 48 * wave;  // this wave's first output channel
        // weight fragments B8_PF k-steps ahead (the loop is unrolled: a register ring with static
        // indices), so the L2 latency of the streamed weights hides behind the MFMAs
        constexpr int B8_PF = 3;
        bf16x8 wr0[B8_PF][3], wr1[B8_PF][3];
        auto load_w = [&](int s, bf16x8 (&d0)[3], bf16x8 (&d1)[3]) {
            const int tap = s / 3, cb = s - 3 * tap;
#pragma unroll
            for (int j = 0; j < 3; j++) {
                const __bf16* wr = w + (int64_t)(nb + 16 * j + r16) * p.ws + tap * B8_C + 64 * cb + 8 * g;
                d0[j] = *(const bf16x8*)wr;
                d1[j] = *(const bf16x8*)(wr + 32);
            }
        };
#pragma unroll
        for (int q = 0; q < B8_PF; q++) load_w(q, wr0[q], wr1[q]);
#pragma unroll
        for (int s = 0; s < 9; s++) {
            const int tap = s / 3, cb = s - 3 * tap;  // k = tap * 192 + 64 cb + ..
            bf16x8 b0[3], b1[3];
#pragma unroll
            for (int j = 0; j < 3; j++) {
                b0[j] = wr0[s % B8_PF][j];
                b1[j] = wr1[s % B8_PF][j];
            }
            if (s + B8_PF < 9) load_w(s + B8_PF, wr0[s % B8_PF], wr1[s % B8_PF]);
#pragma unroll
            for (int i = 0; i < NF; i++) {
                const int yy = vertical ? py[i] + tap - 1 : py[i], xx = vertical ? px[i] : px[i] + tap - 1;
                const bool ok = yy >= 0 && yy < 3 && xx >= 0 && xx < 3;
                const int row = 16 * i + r16 + (vertical ? 3 * (tap - 1) : tap - 1);  // same image: +-3 / +-1
                const char* a = ok ? src + row * B8_RS + (64 * cb + 8 * g) * 2 : Z;
                const bf16x8 a0 = *(const bf16x8*)a;
                const bf16x8 a1 = ok ? *(const bf16x8*)(a + 64) : bf16x8{};
#pragma unroll
                for (int j = 0; j < 3; j++) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1[j], acc[i][j], 0, 0, 0);
                }
            }
        }
        // BN + ReLU -> bf16: stage 0 into the LDS rows of Y, stage 1 into CAT[:, 192:384]
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const int ch = nb + 16 * j + r16;
            const float a = al[ch], b = be[ch];
#pragma unroll
            for (int i = 0; i < NF; i++)
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    const int pix = 16 * i + 4 * g + q;
                    const __bf16 v = (__bf16)relu_bf(fmaf(acc[i][j][q], a, b));
                    if (stage == 0 && pix < NR)
                        *(__bf16*)(Y + pix * B8_RS + ch * 2) = v;
                    else if (pix < 9 * ng)
                        p.cat[((int64_t)n0 * 9 + pix) * (2 * B8_C) + B8_C + ch] = v;
                }
        }
    };
    conv(X, p.wa, p.ala, p.bea, false, 0);  // 1x3 (pad (0, 1))
    __syncthreads();
    conv(Y, p.wb, p.alb, p.beb, true, 1);   // 3x1 (pad (1, 0))
}

// ---------------------------------------------------------------------------------------------
// FaceNet stem head: blobFromImages of the device crops (k_blob's INTER_LINEAR and normalisation,
// facenet.py:179) straight into conv2d_1a (3x3 stride 2, 3 -> 32, BN + ReLU, facenet.py:126): a
// tile of 8 x 16 output pixels computes its 17 x 33 blob patch into LDS (8 bf16 per pixel, the
// blob's NHWC layout: 3 values + 5 zeros) and runs the conv from there, so the 160 x 160 blob never
// goes through HBM.  The conv is k_conv's (conv.hip) for this layer bit for bit: the same
// v_mfma_f32_16x16x32_bf16 chain over k = 0..127 (taps 9..15 zero; K = 72 in two 64-deep k-tiles),
// the same lane -> k mapping, and the same fmaf(acc, alpha, beta) + ReLU epilogue.
constexpr int SH_TH = 8, SH_TW = 16, SH_PH = 2 * SH_TH + 1, SH_PW = 2 * SH_TW + 1;  // patch 17 x 33
constexpr int SH_S = 160, SH_OUT = 79, SH_COUT = 32;
// patch image: per row the 17 even columns, then the 16 odd ones (16 B each): a fragment's lanes
// (output columns tx, input column 2 tx + kx) read consecutive 16-byte slots
constexpr int SH_RS = SH_PW * 16;

struct StemP {
    const uint8_t* frames;
    int F, H, W;
    int64_t fstride, rstride;
    const int32_t* crops;
    const __bf16* w;  // [32][72] (k = tap * 8 + c)
    const float *al, *be;
    __bf16* out;      // [N][79][79][32]
    float mean, scale;
    int tiles_x, tiles_per_img;
};

__device__ inline int sh_slot(int r, int c) { return r * SH_RS + ((c & 1) ? (SH_PW / 2 + 1) * 16 : 0) + (c >> 1) * 16; }

__global__ __launch_bounds__(256) void k_stem_head(StemP p) {
    __shared__ __attribute__((aligned(16))) char P[SH_PH * SH_RS];
    __shared__ __attribute__((aligned(16))) __bf16 E[SH_TH * SH_TW * SH_COUT];
    __shared__ int4 ycf[SH_PH], xcf[SH_PW];  // (s0, s1, c0, c1) per patch row / column; x: edge flag in s1's sign
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int n = blockIdx.x / p.tiles_per_img, t = blockIdx.x - n * p.tiles_per_img;
    const int ty = t / p.tiles_x, oy0 = ty * SH_TH, ox0 = (t - ty * p.tiles_x) * SH_TW;
    int w, h;
    const uint8_t* base = blob_crop(p.frames, p.F, p.H, p.W, p.fstride, p.rstride, p.crops + (int64_t)n * 5, w, h);
    const bool empty = w <= 0 || h <= 0, same = w == SH_S && h == SH_S;
    if (!empty && !same) {
        if (tid < SH_PH) {
            const int d = min(2 * oy0 + tid, SH_S - 1);
            int s0, s1, c0, c1;
            bool e;
            lin_coef(d, h, SH_S, s0, s1, c0, c1, e);
            ycf[tid] = make_int4(s0, s1, c0, c1);
        } else if (tid >= 64 && tid < 64 + SH_PW) {
            const int d = min(2 * ox0 + tid - 64, SH_S - 1);
            int s0, s1, c0, c1;
            bool e;
            lin_coef(d, w, SH_S, s0, s1, c0, c1, e);
            xcf[tid - 64] = make_int4(s0, e ? -1 - s1 : s1, c0, c1);
        }
    }
    // the B operands (weights) meanwhile: lane (channel 16 j + (lane & 15), k = 32 s + 8 (lane >> 4) ..)
    bf16x8 wb[4][2];
#pragma unroll
    for (int s = 0; s < 4; s++)
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const int k = 32 * s + 8 * (lane >> 4);
            wb[s][j] = k < 72 ? *(const bf16x8*)(p.w + (16 * j + (lane & 15)) * 72 + k) : bf16x8{};
        }
    __syncthreads();
    for (int e = tid; e < SH_PH * SH_PW; e += 256) {
        const int r = e / SH_PW, c = e - r * SH_PW;
        const int dy = 2 * oy0 + r, dx = 2 * ox0 + c;
        int v[3] = {0, 0, 0};
        if (!empty && dy < SH_S && dx < SH_S) {
            if (same) {
                const uint8_t* q = base + (int64_t)dy * p.rstride + dx * 3;
                v[0] = q[0], v[1] = q[1], v[2] = q[2];
            } else {
                const int4 yc = ycf[r], xc = xcf[c];
                const bool ex = xc.y < 0;
                const int sx1 = ex ? -1 - xc.y : xc.y;
                const uint8_t* r0 = base + (int64_t)yc.x * p.rstride;
                const uint8_t* r1 = base + (int64_t)yc.y * p.rstride;
#pragma unroll
                for (int ch = 0; ch < 3; ch++) v[ch] = blob_lin(r0, r1, xc.x, sx1, xc.z, xc.w, ex, yc.z, yc.w, ch);
            }
        }
        // (k_blob: swapRB, ((float)v - mean) * scale, bf16; outside the blob: zero)
        bf16x8 px = {};
        if (dy < SH_S && dx < SH_S)
#pragma unroll
            for (int oc = 0; oc < 3; oc++) px[oc] = (__bf16)(((float)v[2 - oc] - p.mean) * p.scale);
        *(bf16x8*)(P + sh_slot(r, c)) = px;
    }
    __syncthreads();
    // wave w: output rows 2 w, 2 w + 1 of the tile (one 16-pixel fragment each)
    f4 acc[2][2];
#pragma unroll
    for (int i = 0; i < 2; i++) acc[i][0] = acc[i][1] = f4{0.f, 0.f, 0.f, 0.f};
    const int tx = lane & 15, g = lane >> 4;
#pragma unroll
    for (int s = 0; s < 4; s++) {
        const int tap = 4 * s + g;
        const int ky = tap / 3, kx = tap - 3 * ky;
#pragma unroll
        for (int i = 0; i < 2; i++) {
            const bf16x8 a = tap < 9 ? *(const bf16x8*)(P + sh_slot(2 * (2 * wave + i) + ky, 2 * tx + kx)) : bf16x8{};
#pragma unroll
            for (int j = 0; j < 2; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wb[s][j], acc[i][j], 0, 0, 0);
        }
    }
    // BN + ReLU -> bf16 staging [128][32] -> 16-byte stores of the in-bounds pixels
#pragma unroll
    for (int j = 0; j < 2; j++) {
        const int ch = 16 * j + (lane & 15);
        const float a = p.al[ch], b = p.be[ch];
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                const int m = 16 * (2 * wave + i) + 4 * g + q;
                E[m * SH_COUT + ch] = (__bf16)relu_bf(fmaf(acc[i][j][q], a, b));
            }
    }
    __syncthreads();
    for (int e = tid; e < SH_TH * SH_TW * SH_COUT / 8; e += 256) {
        const int m = e >> 2, c = e & 3;
        const int oy = oy0 + (m >> 4), ox = ox0 + (m & 15);
        if (oy < SH_OUT && ox < SH_OUT)
            *(bf16x8*)(p.out + (((int64_t)n * SH_OUT + oy) * SH_OUT + ox) * SH_COUT + 8 * c) = *(const bf16x8*)(E + m * SH_COUT + 8 * c);
    }
}

}  // namespace

// one Block17 (bf16 NHWC [N, 8, 8, 896] -> same): weights as FaceNet's layer table holds them
void launch_block17_fused(const void* x, void* y, int N, const void* wm, const float* alm, const float* bem,
                          const void* wa, const float* ala, const float* bea, const void* wb, const float* alb,
                          const float* beb, const void* wo, const float* bo, float scale, hipStream_t st,
                          bool head_only, int ws, int wos) {
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
    p.clk = nullptr;
    p.ws = ws;
    p.wos = wos;
    // (the L2 warm-up covers at most 4 x 256 lines per slice: the strides below keep it there)
    VTF_CHECK(ws >= 896 && ws <= 1024 && ws % 8 == 0 && wos >= 256 && wos <= 384 && wos % 8 == 0, VTF_E_ARG,
              "block17: weight row strides");
    static bool attr = [] {
        VTF_HIP(hipFuncSetAttribute((const void*)k_block17<false>, hipFuncAttributeMaxDynamicSharedMemorySize, K17_LDS));
        VTF_HIP(hipFuncSetAttribute((const void*)k_block17<true>, hipFuncAttributeMaxDynamicSharedMemorySize, K17_LDS));
        return true;
    }();
    (void)attr;
    const char* dbg = std::getenv("VTF_B17_CLK");  // debug: per-stage shader clocks, printed to stderr
    std::vector<unsigned long long> hc;
    if (dbg && std::atoi(dbg)) {
        VTF_HIP(hipMallocAsync((void**)&p.clk, (size_t)N * 5 * 8, st));
        hc.resize((size_t)N * 5);
    }
    if (head_only)
        k_block17<true><<<N, 256, K17_LDS, st>>>(p);
    else
        k_block17<false><<<N, 256, K17_LDS, st>>>(p);
    VTF_HIP(hipGetLastError());
    if (p.clk) {
        VTF_HIP(hipMemcpyAsync(hc.data(), p.clk, hc.size() * 8, hipMemcpyDeviceToHost, st));
        VTF_HIP(hipStreamSynchronize(st));
        VTF_HIP(hipFreeAsync(p.clk, st));
        double d[4] = {0, 0, 0, 0};
        for (int i = 0; i < N; i++)
            for (int k = 0; k < 4; k++) d[k] += (double)(hc[i * 5 + k + 1] - hc[i * 5 + k]) / N;
        fprintf(stderr, "k_block17 cycles per stage (mean over %d workgroups): s1 %.0f s2 %.0f s3 %.0f s4 %.0f\n", N,
                d[0], d[1], d[2], d[3]);
    }
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
        !q.alpha || !q.relu || q.n_split || q.scale != 1.f || q.leaky || q.prelu || q.gelu || q.s3 || q.res_post ||
        q.up2 || q.res_up2 || q.out_f32 || q.f16x || q.out_sp || q.in_sp)
        return false;  // (k_conv_patch applies only fmaf(acc, alpha, beta) then ReLU)
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

namespace vtf {

// FaceNet stem head (bf16): crops of the uint8 frames -> conv2d_1a output [N, 79, 79, 32]
void launch_stem_head(const uint8_t* frames, int F, int H, int W, int64_t fstride, int64_t rstride,
                      const int32_t* d_crops, int N, const void* w, const float* al, const float* be, void* out,
                      hipStream_t st) {
    if (N <= 0) return;
    StemP p;
    p.frames = frames;
    p.F = F;
    p.H = H;
    p.W = W;
    p.fstride = fstride;
    p.rstride = rstride;
    p.crops = d_crops;
    p.w = (const __bf16*)w;
    p.al = al;
    p.be = be;
    p.out = (__bf16*)out;
    p.mean = 127.5f;
    p.scale = 0.0078125f;
    p.tiles_x = (SH_OUT + SH_TW - 1) / SH_TW;
    p.tiles_per_img = p.tiles_x * ((SH_OUT + SH_TH - 1) / SH_TH);
    k_stem_head<<<(unsigned)(N * p.tiles_per_img), 256, 0, st>>>(p);
    VTF_HIP(hipGetLastError());
}

}  // namespace vtf

namespace vtf {

// Block8 branch-1 middle convs (bf16): T1 [N, 3, 3, 192] -> CAT[:, :, :, 192:384]
void launch_block8_mid(const void* t1, void* cat, int N, const void* wa, const float* ala, const float* bea,
                       const void* wb, const float* alb, const float* beb, hipStream_t st, int ws) {
    if (N <= 0) return;
    VTF_CHECK(ws >= 3 * B8_C && ws % 8 == 0, VTF_E_ARG, "block8 middle: weight row stride");
    B8P p;
    p.ws = ws;
    p.t1 = (const __bf16*)t1;
    p.cat = (__bf16*)cat;
    p.wa = (const __bf16*)wa;
    p.wb = (const __bf16*)wb;
    p.ala = ala;
    p.bea = bea;
    p.alb = alb;
    p.beb = beb;
    p.N = N;
    // images per workgroup (VTF_B8_G: 1, 3 or 7, experiments)
    static const int gsel = [] {
        const char* e = std::getenv("VTF_B8_G");
        return e ? std::atoi(e) : 1;
    }();
    if (gsel == 7)
        k_block8_mid<7><<<(unsigned)((N + 6) / 7), 256, 0, st>>>(p);
    else if (gsel == 3)
        k_block8_mid<3><<<(unsigned)((N + 2) / 3), 256, 0, st>>>(p);
    else
        k_block8_mid<1><<<(unsigned)N, 256, 0, st>>>(p);
    VTF_HIP(hipGetLastError());
}

}  // namespace vtf

// Implicit-GEMM convolution on MFMA for gfx950 (NHWC activations).
//
// Replaces the torch.nn.Conv2d + BatchNorm2d + ReLU stacks of ConvUnit
// (src/videotofaces/backbones/basic.py:5-45) and the residual tails of Block35/17/8
// (src/videotofaces/encoders/facenet.py:14-81) -- the encoder conv path.
//   GEMM view: M = N*OH*OW output pixels, N = Cout, K = KH*KW*Cin (k = (kh, kw, ci)).
//   A = im2col gathered on the fly from NHWC input (16-B vectors along ci),
//   B = weights [Cout][K] (host re-layout), C -> fused epilogue -> NHWC output slice
//   (channel offset + stride, so Inception concats are free).
// Three operand modes from one template:
//   fp32: v_mfma_f32_16x16x4_f32  (exact fp32 products, parity mode, 1e-4 vs the reference)
//   f16x: fp32 operands split at LDS staging into x0 + x1 * 2^-11 fp16 planes, three
//         v_mfma_f32_16x16x32_f16 per 32-deep step (fp32-grade products; callers guarantee or
//         guard the fp16 range -- ConvParams::f16x / ovf)
//   bf16: v_mfma_f32_16x16x32_bf16 (bf16 operands/activations, fp32 accumulate; perf mode)
// Tile: BM x BN per 256-thread workgroup (2x2 waves, each (BM/2)x(BN/2) = 16x16 fragments),
// BK-deep K steps, global->register prefetch of step k+1 while step k runs on MFMA from LDS;
// split-K over blockIdx.z for grids that cannot fill the chip.  Epilogue staged through LDS:
// each thread finishes 8 consecutive channels of a row (16/32-byte residual loads / stores).
#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <unordered_map>

#include "common.hpp"
#include "conv.hpp"
#include "conv_dev.hpp"

// timing-only staging switches (scripts/ab_xdbg.sh): build with -DVTF_CONV_XDBG=1
#ifndef VTF_CONV_XDBG
#define VTF_CONV_XDBG 0
#endif

namespace vtf {

template <typename T, int BM, int BN, int BK, bool SPLIT, bool X = false>
__global__ __launch_bounds__(256) void k_conv(ConvParams p) {
    using vec = typename VecT<T>::type;
    constexpr int V = VecT<T>::V;
    // row pads chosen for conflict-free fragment reads.  ds_read_b128 (bf16, split) serves
    // 16-lane groups {0-3,12-15,20-27}, ... with bank = dword mod 64: a 144-B bf16 row / 80-B
    // split row put two lanes of a group on one bank (2 LDS cycles per read), 160 B / 96 B do
    // not.  ds_read_b32 (fp32: rows lane&15, k = lane>>4) serves lanes 0-31 with bank = dword
    // mod 32: a 36-float row maps rows r and r+8 to one bank, a 34-float row (2r + k) does not
    constexpr int PAD = sizeof(T) == 2 ? 16 : 2;
    constexpr int LDA = BK + PAD;
    constexpr int KV = BK / V;                // vectors per tile row
    constexpr int RA = BM * KV / 256;         // A vectors per thread
    constexpr int RB = BN * KV / 256;         // B vectors per thread
    static_assert(RA >= 1 && RB >= 1 && (256 % KV) == 0, "tile config");
    static_assert(!X || (sizeof(T) == 4 && BK == 32), "split-fp16 mode: fp32 operands, one 32-deep step");
    constexpr int WM = BM / 2, WN = BN / 2, FM = WM / 16, FN = WN / 16;
    // X: fp16 split planes [2][rows][LDH] (row stride 96 B: 16-B aligned, conflict-free reads)
    constexpr int LDH = BK + 16;
    constexpr int A_BYTES = X ? 2 * BM * LDH * 2 : BM * LDA * (int)sizeof(T);
    constexpr int B_BYTES = X ? 2 * BN * LDH * 2 : BN * LDA * (int)sizeof(T);
    // the operand tiles, reused after the K loop as the fp32 output tile of the staged epilogue
    constexpr int LDE = BN + 4;
    constexpr int E_BYTES = SPLIT ? 0 : BM * LDE * 4;
    constexpr int SM_BYTES = A_BYTES + B_BYTES > E_BYTES ? A_BYTES + B_BYTES : E_BYTES;
    __shared__ __attribute__((aligned(16))) char smem[SM_BYTES];
    char* As_raw = smem;
    char* Bs_raw = smem + A_BYTES;
    T* As = (T*)As_raw;
    T* Bs = (T*)Bs_raw;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    // XCD-aware tile order: workgroups are dealt to the 8 XCDs round-robin in dispatch order
    // (linear id % 8), each XCD with its own L2.  Re-number so that every XCD owns one
    // contiguous run of tiles and walks it in groups of group_m M-tiles x all N-tiles: the A
    // row-blocks and B column-blocks its resident workgroups share stay in its L2.  (Placement
    // only affects speed; any bijection is correct.)
    int tile_m = blockIdx.x, tile_n = blockIdx.y;
    if (p.group_m > 0) {
        const int gx = gridDim.x, gy = gridDim.y;
        const int lin = blockIdx.x + gx * blockIdx.y, total = gx * gy;
        const int xcd = lin & 7, loc = lin >> 3, per = total >> 3, rem = total & 7;
        const int L = xcd < rem ? xcd * (per + 1) + loc : rem * (per + 1) + (xcd - rem) * per + loc;
        const int span = p.group_m * gy;
        const int first = (L / span) * p.group_m;
        const int gsz = min(gx - first, p.group_m);
        tile_m = first + (L % span) % gsz;
        tile_n = (L % span) / gsz;
    }
    const int64_t m0 = (int64_t)tile_m * BM;
    const int n0 = tile_n * BN;
    const T* __restrict__ in = (const T*)p.in;
    const T* __restrict__ wt = (const T*)p.w;
    const int ics = p.in_cstride ? p.in_cstride : p.Cin;

    // per-thread A rows and the thread's k-vector position
    const int kv = tid % KV;
    int64_t a_base[RA];
    int a_ih0[RA], a_iw0[RA];
    bool a_ok[RA];
#pragma unroll
    for (int r = 0; r < RA; r++) {
        int row = (tid + 256 * r) / KV;
        int64_t m = m0 + row;
        a_ok[r] = m < p.M;
        int64_t mm = a_ok[r] ? m : 0;
        int ow = (int)(mm % p.OW);
        int64_t t = mm / p.OW;
        int oh = (int)(t % p.OH);
        int n = (int)(t / p.OH);
        a_base[r] = (int64_t)n * p.H * p.W * ics;
        a_ih0[r] = oh * p.sh - p.ph;
        a_iw0[r] = ow * p.sw - p.pw;
    }
    // split-K slice z covers k-tiles [kt0, kt1)
    const int KT_all = (p.K + BK - 1) / BK;
    const int kt0 = SPLIT ? (int)((int64_t)blockIdx.z * KT_all / p.split) : 0;
    const int kt1 = SPLIT ? (int)((int64_t)(blockIdx.z + 1) * KT_all / p.split) : KT_all;
    int k = kt0 * BK + kv * V;
    int ci = k % p.Cin, kw_ = (k / p.Cin) % p.KW, kh_ = (k / p.Cin) / p.KW;

    vec ra[RA], rb[RB];
    auto load_tile = [&](int kcur, int ci_, int kw0, int kh0) {
#if VTF_CONV_XDBG
        if (X && (p.xdbg & 2)) {
#pragma unroll
            for (int r = 0; r < RA; r++) ra[r] = vec{};
#pragma unroll
            for (int r = 0; r < RB; r++) rb[r] = vec{};
            return;
        }
#endif
#pragma unroll
        for (int r = 0; r < RA; r++) {
            vec v = {};
            int ih = a_ih0[r] + kh0, iw = a_iw0[r] + kw0;
            if (a_ok[r] && kcur < p.K && ih >= 0 && ih < p.H && iw >= 0 && iw < p.W)
                v = *(const vec*)(in + a_base[r] + ((int64_t)ih * p.W + iw) * ics + ci_);
            ra[r] = v;
        }
#pragma unroll
        for (int r = 0; r < RB; r++) {
            int row = (tid + 256 * r) / KV;
            int co = n0 + row;
            vec v = {};
            if (co < p.Cout && kcur < p.K) v = *(const vec*)(wt + (int64_t)co * p.K + kcur);
            rb[r] = v;
        }
    };
    auto store_tile = [&]() {
        if constexpr (X) {
            typedef __attribute__((ext_vector_type(4))) _Float16 h4;
            auto put = [&](char* base, int rows, int row, const vec& v) {
                h4 x0, x1;
                float mx = 0.f;
#if VTF_CONV_XDBG
                if (p.xdbg & 1) {
#pragma unroll
                    for (int e = 0; e < 4; e++) x0[e] = x1[e] = (_Float16)to_f(v[e]);
                } else
#endif
                {
#pragma unroll
                    for (int e = 0; e < 4; e++) {
                        x0[e] = (_Float16)to_f(v[e]);
                        x1[e] = (_Float16)((to_f(v[e]) - (float)x0[e]) * 2048.f);
                        mx = fmaxf(mx, fabsf(to_f(v[e])));
                    }
                }
                // also catches NaN; one atomic per wave, not per lane
                if (p.ovf && __ballot(!(mx < 16384.f)) && __lane_id() == 0) atomicOr(p.ovf, 1);
                _Float16* h = (_Float16*)base;
                *(h4*)(h + row * LDH + kv * 4) = x0;
                *(h4*)(h + rows * LDH + row * LDH + kv * 4) = x1;
            };
#pragma unroll
            for (int r = 0; r < RA; r++) put(As_raw, BM, (tid + 256 * r) / KV, ra[r]);
#pragma unroll
            for (int r = 0; r < RB; r++) put(Bs_raw, BN, (tid + 256 * r) / KV, rb[r]);
        } else {
            // fp32 rows of 34 floats are 8-B aligned only: two 8-byte stores per vector
            auto st = [&](T* dst, const vec& v) {
                if constexpr (LDA % V == 0) {
                    *(vec*)dst = v;
                } else {
                    typedef __attribute__((ext_vector_type(2))) float f32x2;
                    *(f32x2*)dst = f32x2{to_f(v[0]), to_f(v[1])};
                    *(f32x2*)(dst + 2) = f32x2{to_f(v[2]), to_f(v[3])};
                }
            };
#pragma unroll
            for (int r = 0; r < RA; r++) st(As + ((tid + 256 * r) / KV) * LDA + kv * V, ra[r]);
#pragma unroll
            for (int r = 0; r < RB; r++) st(Bs + ((tid + 256 * r) / KV) * LDA + kv * V, rb[r]);
        }
    };
    auto advance = [&]() {
        k += BK;
        ci += BK;
        while (ci >= p.Cin) {
            ci -= p.Cin;
            if (++kw_ == p.KW) {
                kw_ = 0;
                kh_++;
            }
        }
    };

    f32x4 acc[FM][FN], accx[X ? FM : 1][X ? FN : 1];
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    if constexpr (X) {
#pragma unroll
        for (int i = 0; i < FM; i++)
#pragma unroll
            for (int j = 0; j < FN; j++) accx[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    }

    const int KT = kt1 - kt0;
    load_tile(k, ci, kw_, kh_);
    store_tile();
    __syncthreads();
    for (int kt = 0; kt < KT; kt++) {
        if (kt + 1 < KT) {
            advance();
            load_tile(k, ci, kw_, kh_);
        }
        const T* Aw = As + (wm * WM + (lane & 15)) * LDA;
        const T* Bw = Bs + (wn * WN + (lane & 15)) * LDA;
        if constexpr (X) {
            // x*w = x0 w0 + 2^-11 (x0 w1 + x1 w0): main and cross products in separate accumulators
            typedef __attribute__((ext_vector_type(8))) _Float16 h8;
            const _Float16* A0 = (const _Float16*)As_raw + (wm * WM + (lane & 15)) * LDH + 8 * (lane >> 4);
            const _Float16* B0 = (const _Float16*)Bs_raw + (wn * WN + (lane & 15)) * LDH + 8 * (lane >> 4);
            h8 a0[FM], a1[FM], b0[FN], b1[FN];
#pragma unroll
            for (int i = 0; i < FM; i++) {
                a0[i] = *(const h8*)(A0 + i * 16 * LDH);
                a1[i] = *(const h8*)(A0 + BM * LDH + i * 16 * LDH);
            }
#pragma unroll
            for (int j = 0; j < FN; j++) {
                b0[j] = *(const h8*)(B0 + j * 16 * LDH);
                b1[j] = *(const h8*)(B0 + BN * LDH + j * 16 * LDH);
            }
#pragma unroll
            for (int i = 0; i < FM; i++)
#pragma unroll
                for (int j = 0; j < FN; j++) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0[i], b0[j], acc[i][j], 0, 0, 0);
                    accx[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0[i], b1[j], accx[i][j], 0, 0, 0);
                    accx[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[i], b0[j], accx[i][j], 0, 0, 0);
                }
        } else if constexpr (sizeof(T) == 2) {
#pragma unroll
            for (int ks = 0; ks < BK; ks += 32) {
                bf16x8 af[FM], bfr[FN];
#pragma unroll
                for (int i = 0; i < FM; i++) af[i] = *(const bf16x8*)(Aw + i * 16 * LDA + ks + 8 * (lane >> 4));
#pragma unroll
                for (int j = 0; j < FN; j++) bfr[j] = *(const bf16x8*)(Bw + j * 16 * LDA + ks + 8 * (lane >> 4));
#pragma unroll
                for (int i = 0; i < FM; i++)
#pragma unroll
                    for (int j = 0; j < FN; j++)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
            }
        } else {
#pragma unroll
            for (int ks = 0; ks < BK; ks += 4) {
                float af[FM], bfr[FN];
#pragma unroll
                for (int i = 0; i < FM; i++) af[i] = to_f(Aw[i * 16 * LDA + ks + (lane >> 4)]);
#pragma unroll
                for (int j = 0; j < FN; j++) bfr[j] = to_f(Bw[j * 16 * LDA + ks + (lane >> 4)]);
#pragma unroll
                for (int i = 0; i < FM; i++)
#pragma unroll
                    for (int j = 0; j < FN; j++)
                        acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x4f32(af[i], bfr[j], acc[i][j], 0, 0, 0);
            }
        }
        __syncthreads();
        if (kt + 1 < KT) {
            store_tile();
            __syncthreads();
        }
    }

    if constexpr (X) {
#pragma unroll
        for (int i = 0; i < FM; i++)
#pragma unroll
            for (int j = 0; j < FN; j++) acc[i][j] = acc[i][j] + accx[i][j] * 0.00048828125f;
    }
    // staged epilogue: the accumulator tile goes through LDS so every thread finishes 8
    // consecutive channels of a row -- 16-byte residual loads and output stores instead of
    // 2-byte accesses scattered over 4 rows per instruction
    if constexpr (!SPLIT) {
        const bool vec_ok = (p.Cout % 8 == 0) && (p.out_cstride % 8 == 0) && (p.out_coff % 8 == 0) &&
                            (!p.res || p.res_cstride % 8 == 0) &&
                            (!p.n_split || (p.n_split % 8 == 0 && p.out2_cstride % 8 == 0 && p.out2_coff % 8 == 0));
        if (vec_ok) {
            __syncthreads();  // every wave is done with the operand tiles
            float* E = (float*)smem;
#pragma unroll
            for (int j = 0; j < FN; j++)
#pragma unroll
                for (int i = 0; i < FM; i++)
#pragma unroll
                    for (int q = 0; q < 4; q++)
                        E[(wm * WM + i * 16 + 4 * (lane >> 4) + q) * LDE + wn * WN + j * 16 + (lane & 15)] = acc[i][j][q];
            __syncthreads();
            constexpr int G = BN / 8;  // 8-channel groups per row
            static_assert(256 % G == 0, "epilogue groups");
            const int g = tid % G, c0 = n0 + 8 * g;
            if (c0 < p.Cout) {
                float b8[8], al8[8], be8[8], pr8[8];
#pragma unroll
                for (int e = 0; e < 8; e++) {
                    b8[e] = p.bias ? p.bias[c0 + e] : 0.f;
                    al8[e] = p.alpha ? p.alpha[c0 + e] : 1.f;
                    be8[e] = p.alpha ? p.beta[c0 + e] : 0.f;
                    pr8[e] = p.prelu ? p.prelu[c0 + e] : 0.f;
                }
                for (int r = tid / G; r < BM; r += 256 / G) {
                    const int64_t m = m0 + r;
                    if (m >= p.M) break;
                    const f32x4 lo = *(const f32x4*)(E + r * LDE + 8 * g), hi = *(const f32x4*)(E + r * LDE + 8 * g + 4);
                    float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
                    conv_epilogue8<T>(p, m, c0, v, b8, al8, be8, pr8);
                }
            }
            return;
        }
    }
    // epilogue: C layout col = lane & 15, row = 4 * (lane >> 4) + i.  Per 16-column fragment,
    // the residual elements are loaded first (one batch of loads in flight, not one round trip
    // per output behind the previous store), then the outputs are finished and stored.
#pragma unroll
    for (int j = 0; j < FN; j++) {
        const int c = n0 + wn * WN + j * 16 + (lane & 15);
        if constexpr (SPLIT) {
            if (c < p.Cout) {
#pragma unroll
                for (int i = 0; i < FM; i++)
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int64_t m = m0 + wm * WM + i * 16 + 4 * (lane >> 4) + q;
                        if (m < p.M) p.ws[((int64_t)blockIdx.z * p.M + m) * p.Cout + c] = acc[i][j][q];
                    }
            }
        } else {
            float rv[FM][4];
            if (p.res) {
                const T* __restrict__ res = (const T*)p.res;
                const int cc = min(c, p.Cout - 1);
#pragma unroll
                for (int i = 0; i < FM; i++)
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int64_t m = min(m0 + wm * WM + i * 16 + 4 * (lane >> 4) + q, p.M - 1);
                        rv[i][q] = to_f(res[res_index(p, m, cc)]);
                    }
            }
            if (c < p.Cout) {
                const float bias = p.bias ? p.bias[c] : 0.f;
                const float al = p.alpha ? p.alpha[c] : 1.f;
                const float be = p.alpha ? p.beta[c] : 0.f;
                const float pr = p.prelu ? p.prelu[c] : 0.f;
#pragma unroll
                for (int i = 0; i < FM; i++)
#pragma unroll
                    for (int q = 0; q < 4; q++) {
                        const int64_t m = m0 + wm * WM + i * 16 + 4 * (lane >> 4) + q;
                        if (m < p.M) conv_epilogue<T>(p, m, c, acc[i][j][q], bias, al, be, pr, p.res ? rv[i][q] : 0.f);
                    }
            }
        }
    }
}

// split-K: sum the partial slabs in slice order (deterministic), then the fused epilogue
template <typename T>
__global__ void k_conv_splitk_epi(ConvParams p) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= p.M * p.Cout) return;
    const int c = (int)(i % p.Cout);
    const int64_t m = i / p.Cout;
    float v = 0.f;
    for (int z = 0; z < p.split; z++) v += p.ws[((int64_t)z * p.M + m) * p.Cout + c];
    const float rv = p.res ? to_f(((const T*)p.res)[res_index(p, m, c)]) : 0.f;
    conv_epilogue<T>(p, m, c, v, p.bias ? p.bias[c] : 0.f, p.alpha ? p.alpha[c] : 1.f, p.alpha ? p.beta[c] : 0.f,
                     p.prelu ? p.prelu[c] : 0.f, rv);
}

// per-stream split-K workspace (lanes run concurrently on their own streams); grows x1.5, never
// shrinks; an outgrown buffer is retired rather than freed (hipFree would synchronize the device
// and queued kernels may still use it) -- bounded by the geometric growth, process lifetime
static float* splitk_workspace(hipStream_t st, size_t bytes) {
    static std::mutex mu;
    // keyed by (device, stream): the null stream of two devices is two different queues
    static std::map<std::pair<int, hipStream_t>, std::pair<float*, size_t>> ws;
    static std::vector<float*> retired;
    const int dev = stream_device(st);
    std::lock_guard<std::mutex> g(mu);
    auto& e = ws[{dev, st}];
    if (e.second < bytes) {
        if (e.first) retired.push_back(e.first);
        e.first = nullptr;
        e.second = 0;
        const size_t b = bytes + bytes / 2;
        VTF_HIP(hipMalloc((void**)&e.first, b));
        e.second = b;
    }
    return e.first;
}

// bf16 grids of 64-row tiles below this many workgroups per CU use 32-row tiles instead: each
// workgroup's K loop is load-latency bound (one register stage), so more resident workgroups per
// CU is what hides it (VTF_CONV_BF16_SMALL = the threshold in workgroups per CU; 0 disables)
static int conv_small_wg_per_cu() {
    static int v = [] {
        const char* e = std::getenv("VTF_CONV_BF16_SMALL");
        return e ? std::atoi(e) : 3;
    }();
    return v;
}
static int device_cus() {
    static int cus = [] {
        int dev = 0, n = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        return n;
    }();
    return cus;
}

// M-tile group height of the XCD-aware tile order (VTF_CONV_GROUP_M overrides; 0 = plain)
static int conv_group_m() {
    static int g = [] {
        const char* e = std::getenv("VTF_CONV_GROUP_M");
        return e ? std::atoi(e) : 8;
    }();
    return g;
}

// split factor: grids far below the CU count (FaceNet Block17/Block8, YOLO/R-CNN deep stages at
// small batch) are split along K into up to 8 slices so ~2 workgroups land on every CU. bf16
// (perf) mode only: the fp32 parity mode keeps the single-pass summation order.
bool splitk_disabled() {
    const char* e = std::getenv("VTF_NO_SPLITK");
    return e && std::atoi(e) != 0;
}

static int pick_split(int64_t tiles, int KT, bool bf16, bool fp32_split) {
    // bf16: grids below 192 tiles; fp32 callers that accept a slice-order reduction
    // (split_fp32: ONet's dense layer, 120 tiles of K = 1152: 72 -> 51 us with the epilogue
    // kernel; RNet's 196 tiles of K = 576 measured slower split) below 160
    // (VTF_SPLIT_TILES / VTF_SPLIT_WG: the bf16 tile threshold and workgroup target, experiments)
    static const int thr = [] {
        const char* e = std::getenv("VTF_SPLIT_TILES");
        return e ? std::atoi(e) : 192;
    }();
    static const int tgt = [] {
        const char* e = std::getenv("VTF_SPLIT_WG");
        return e ? std::atoi(e) : 512;
    }();
    if (!(bf16 || fp32_split) || tiles >= (bf16 ? thr : 160) || KT < 8 || splitk_disabled()) return 1;
    int s = (int)std::min<int64_t>(8, ((bf16 ? tgt : 512) + tiles - 1) / tiles);
    s = std::min(s, KT / 4);
    return s < 2 ? 1 : s;
}

template <typename T, int BM, int BN, int BK>
static void launch_tile(const ConvParams& p0, hipStream_t st) {
    ConvParams p = p0;
    const int64_t gx = cdiv(p.M, BM), gy = cdiv(p.Cout, BN);
    const int KT = (p.K + BK - 1) / BK;
    p.split = pick_split(gx * gy, KT, sizeof(T) == 2, sizeof(T) == 4 && p.split_fp32);
    p.ws = nullptr;
    if (p.split > 1) p.ws = splitk_workspace(st, (size_t)p.split * p.M * p.Cout * sizeof(float));
    p.group_m = conv_group_m();
#if VTF_CONV_XDBG
    static const int xdbg = [] {
        const char* e = std::getenv("VTF_CONV_XDBG");
        return e ? std::atoi(e) : 0;
    }();
    p.xdbg = p.f16x ? xdbg : 0;
#endif
    dim3 g((unsigned)gx, (unsigned)gy, (unsigned)p.split);
    if (p.split > 1) {
        if constexpr (sizeof(T) == 4) {
            if (p.f16x)
                k_conv<T, BM, BN, BK, true, true><<<g, 256, 0, st>>>(p);
            else
                k_conv<T, BM, BN, BK, true><<<g, 256, 0, st>>>(p);
        } else {
            k_conv<T, BM, BN, BK, true><<<g, 256, 0, st>>>(p);
        }
        const int64_t n = p.M * p.Cout;
        k_conv_splitk_epi<T><<<(unsigned)cdiv(n, 256), 256, 0, st>>>(p);
        return;
    }
    if constexpr (sizeof(T) == 4) {
        if (p.f16x) {
            k_conv<T, BM, BN, BK, false, true><<<g, 256, 0, st>>>(p);
            return;
        }
    }
    k_conv<T, BM, BN, BK, false><<<g, 256, 0, st>>>(p);
}

template <typename T>
static void launch_t(const ConvParams& p, hipStream_t st) {
    // bf16: 64-row tiles throughout -- measured on FaceNet (batch 128), twice the workgroups of
    // 128-row tiles hide more load latency than the larger tiles save in operand traffic
    // (forward 2.82 -> 2.67 ms); the per-output k order does not depend on the tile shape.
    // fp32 (parity) keeps 128-row tiles.
    if constexpr (sizeof(T) == 2) {
        const int BN = p.Cout <= 32 ? 32 : 64;
        const int64_t wg64 = (int64_t)cdiv(p.M, 64) * cdiv(p.Cout, BN);
        if (wg64 < (int64_t)conv_small_wg_per_cu() * device_cus()) {
            if (BN == 32)
                launch_tile<T, 32, 32, 64>(p, st);
            else
                launch_tile<T, 32, 64, 64>(p, st);
            return;
        }
    }
    if (p.Cout <= 32) {
        if constexpr (sizeof(T) == 2)
            launch_tile<T, 64, 32, 64>(p, st);
        else
            launch_tile<T, 128, 32, 32>(p, st);
    } else {
        if constexpr (sizeof(T) == 2)
            launch_tile<T, 64, 64, 64>(p, st);
        else
            launch_tile<T, 128, 64, 32>(p, st);
    }
}

void launch_conv(const ConvParams& p, bool bf16, hipStream_t st) {
    if (p.M <= 0) return;
    VTF_CHECK(p.Cin % 8 == 0, VTF_E_ARG, "conv: Cin must be a multiple of 8 (pad the input)");
    VTF_CHECK(p.in_cstride == 0 || (p.in_cstride >= p.Cin && p.in_cstride % 8 == 0), VTF_E_ARG,
              "conv: bad input channel stride");
    VTF_CHECK(!p.res_up2 || (p.OH % 2 == 0 && p.OW % 2 == 0), VTF_E_ARG, "conv: half-resolution residual needs even OH/OW");
    VTF_CHECK(!p.n_split || (p.out2 && p.n_split > 0 && p.n_split < p.Cout && !p.up2 && !p.out_f32), VTF_E_ARG,
              "conv: output split needs out2, 0 < n_split < Cout, plain layout");
    // bf16 convs go to the LDS-DMA kernel (conv_dma.hip) when their channel counts allow it
    // (VTF_CONV_DMA=0 keeps k_conv: A/B timing)
    static const bool dma = [] {
        const char* e = std::getenv("VTF_CONV_DMA");
        return !(e && std::atoi(e) == 0);
    }();
    if (bf16 && dma && conv_dma_choice_bf16(p) != 0) {
        launch_conv_dma(p, true, st);
        return;
    }
    if (bf16)
        launch_t<__bf16>(p, st);
    else
        launch_t<float>(p, st);
}

// ---------------------------------------------------------------- maxpool 3x3 / 2, no padding (NHWC)
template <typename T>
__global__ void k_maxpool(const T* __restrict__ in, int N, int H, int W, int C, int OH, int OW, T* __restrict__ out,
                          int out_cstride, int out_coff) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t tot = (int64_t)N * OH * OW * C;
    if (i >= tot) return;
    int c = (int)(i % C);
    int64_t t = i / C;
    int ow = (int)(t % OW);
    t /= OW;
    int oh = (int)(t % OH);
    int n = (int)(t / OH);
    float m = -3.402823466e38f;
    for (int dy = 0; dy < 3; dy++)
        for (int dx = 0; dx < 3; dx++)
            m = fmaxf(m, to_f(in[(((int64_t)n * H + 2 * oh + dy) * W + 2 * ow + dx) * C + c]));
    out[(((int64_t)n * OH + oh) * OW + ow) * out_cstride + out_coff + c] = from_f<T>(m);
}

// bf16, 8 channels per thread (C, out_cstride, out_coff multiples of 8): 16-byte loads and stores
// (the max is exact, so the same bits as k_maxpool)
__global__ void k_maxpool_bf16x8(const __bf16* __restrict__ in, int N, int H, int W, int C, int OH, int OW,
                                 __bf16* __restrict__ out, int out_cstride, int out_coff) {
    const int C8 = C >> 3;
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)N * OH * OW * C8) return;
    const int c8 = (int)(i % C8);
    int64_t t = i / C8;
    const int ow = (int)(t % OW);
    t /= OW;
    const int oh = (int)(t % OH);
    const int n = (int)(t / OH);
    float m[8];
#pragma unroll
    for (int e = 0; e < 8; e++) m[e] = -3.402823466e38f;
    const __bf16* src = in + (((int64_t)n * H + 2 * oh) * W + 2 * ow) * C + 8 * c8;
#pragma unroll
    for (int dy = 0; dy < 3; dy++)
#pragma unroll
        for (int dx = 0; dx < 3; dx++) {
            const bf16x8 v = *(const bf16x8*)(src + ((int64_t)dy * W + dx) * C);
#pragma unroll
            for (int e = 0; e < 8; e++) m[e] = fmaxf(m[e], (float)v[e]);
        }
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; e++) o[e] = (__bf16)m[e];
    *(bf16x8*)(out + (((int64_t)n * OH + oh) * OW + ow) * out_cstride + out_coff + 8 * c8) = o;
}

void launch_maxpool(const void* in, int N, int H, int W, int C, void* out, int out_cstride, int out_coff, bool bf16,
                    hipStream_t st) {
    int OH = (H - 3) / 2 + 1, OW = (W - 3) / 2 + 1;
    int64_t tot = (int64_t)N * OH * OW * C;
    if (bf16 && C % 8 == 0 && out_cstride % 8 == 0 && out_coff % 8 == 0) {
        k_maxpool_bf16x8<<<cdiv(tot / 8, 256), 256, 0, st>>>((const __bf16*)in, N, H, W, C, OH, OW, (__bf16*)out,
                                                             out_cstride, out_coff);
        return;
    }
    if (bf16)
        k_maxpool<__bf16><<<cdiv(tot, 256), 256, 0, st>>>((const __bf16*)in, N, H, W, C, OH, OW, (__bf16*)out,
                                                           out_cstride, out_coff);
    else
        k_maxpool<float><<<cdiv(tot, 256), 256, 0, st>>>((const float*)in, N, H, W, C, OH, OW, (float*)out,
                                                          out_cstride, out_coff);
}

// ---------------------------------------------------------------- maxpool k/s with ceil_mode (NHWC fp32)
// one thread per (output pixel, 4 channels): 16-B loads/stores along C (C % 4 == 0)
__global__ void k_maxpool_ks(const float* __restrict__ in, int N, int H, int W, int C, int k, int s, int OH, int OW,
                             float* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int C4 = C >> 2;
    int64_t tot = (int64_t)N * OH * OW * C4;
    if (i >= tot) return;
    int c4 = (int)(i % C4);
    int64_t t = i / C4;
    int ow = (int)(t % OW);
    t /= OW;
    int oh = (int)(t % OH);
    int n = (int)(t / OH);
    f32x4 m = {-3.402823466e38f, -3.402823466e38f, -3.402823466e38f, -3.402823466e38f};
    const f32x4* src = (const f32x4*)in + (int64_t)n * H * W * C4 + c4;
    for (int dy = 0; dy < k; dy++) {
        int y = oh * s + dy;
        if (y >= H) break;
        for (int dx = 0; dx < k; dx++) {
            int x = ow * s + dx;
            if (x >= W) break;
            f32x4 v = src[((int64_t)y * W + x) * C4];
            m.x = fmaxf(m.x, v.x);
            m.y = fmaxf(m.y, v.y);
            m.z = fmaxf(m.z, v.z);
            m.w = fmaxf(m.w, v.w);
        }
    }
    ((f32x4*)out)[i] = m;
}

static int pool_out(int L, int k, int s, bool ceil_mode) {
    // torch pooling_output_shape with padding 0, dilation 1
    int o = ((L - k + (ceil_mode ? s - 1 : 0)) / s) + 1;
    if (ceil_mode && (o - 1) * s >= L) o--;
    return o;
}

// the same pool writing the split-pair layout (gemm_x3.hpp) for a split-mode conv; a value beyond
// the fp16 range raises *ovf
__global__ void k_maxpool_ks_sp(const float* __restrict__ in, int N, int H, int W, int C, int k, int s, int OH, int OW,
                                char* __restrict__ out, int* __restrict__ ovf) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int C4 = C >> 2;
    int64_t tot = (int64_t)N * OH * OW * C4;
    bool bad = false;
    if (i < tot) {
        int c4 = (int)(i % C4);
        int64_t t = i / C4;
        int ow = (int)(t % OW);
        t /= OW;
        int oh = (int)(t % OH);
        int n = (int)(t / OH);
        f32x4 m = {-3.402823466e38f, -3.402823466e38f, -3.402823466e38f, -3.402823466e38f};
        const f32x4* src = (const f32x4*)in + (int64_t)n * H * W * C4 + c4;
        for (int dy = 0; dy < k; dy++) {
            int y = oh * s + dy;
            if (y >= H) break;
            for (int dx = 0; dx < k; dx++) {
                int x = ow * s + dx;
                if (x >= W) break;
                f32x4 v = src[((int64_t)y * W + x) * C4];
                m.x = fmaxf(m.x, v.x);
                m.y = fmaxf(m.y, v.y);
                m.z = fmaxf(m.z, v.z);
                m.w = fmaxf(m.w, v.w);
            }
        }
        sp_store4(out + (i / C4) * (int64_t)C * 4, 4 * c4, m.x, m.y, m.z, m.w, bad);
    }
    if (__ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(ovf, 1);
}

void launch_maxpool_ks_sp(const float* in, int N, int H, int W, int C, int k, int s, bool ceil_mode, void* out, int& OH,
                          int& OW, int* ovf, hipStream_t st) {
    OH = pool_out(H, k, s, ceil_mode);
    OW = pool_out(W, k, s, ceil_mode);
    VTF_CHECK(C % 8 == 0, VTF_E_ARG, "maxpool (split pairs): C must be a multiple of 8");
    int64_t tot = (int64_t)N * OH * OW * (C / 4);
    if (tot > 0) k_maxpool_ks_sp<<<cdiv(tot, 256), 256, 0, st>>>(in, N, H, W, C, k, s, OH, OW, (char*)out, ovf);
}


void launch_maxpool_ks(const float* in, int N, int H, int W, int C, int k, int s, bool ceil_mode, float* out,
                       int& OH, int& OW, hipStream_t st) {
    OH = pool_out(H, k, s, ceil_mode);
    OW = pool_out(W, k, s, ceil_mode);
    VTF_CHECK(C % 4 == 0, VTF_E_ARG, "maxpool: C must be a multiple of 4");
    int64_t tot = (int64_t)N * OH * OW * (C / 4);
    if (tot > 0) k_maxpool_ks<<<cdiv(tot, 256), 256, 0, st>>>(in, N, H, W, C, k, s, OH, OW, out);
}

// ---------------------------------------------------------------- NCHW fp32 -> NHWC (C padded to Cp)
template <typename T>
__global__ void k_nchw_to_nhwc(const float* __restrict__ in, int N, int C, int H, int W, int Cp, T* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t tot = (int64_t)N * H * W * Cp;
    if (i >= tot) return;
    int c = (int)(i % Cp);
    int64_t t = i / Cp;
    int w = (int)(t % W);
    t /= W;
    int h = (int)(t % H);
    int n = (int)(t / H);
    float v = c < C ? in[(((int64_t)n * C + c) * H + h) * W + w] : 0.f;
    out[i] = from_f<T>(v);
}

void launch_nchw_to_nhwc(const float* in, int N, int C, int H, int W, int Cp, void* out, bool bf16, hipStream_t st) {
    int64_t tot = (int64_t)N * H * W * Cp;
    if (bf16)
        k_nchw_to_nhwc<__bf16><<<cdiv(tot, 256), 256, 0, st>>>(in, N, C, H, W, Cp, (__bf16*)out);
    else
        k_nchw_to_nhwc<float><<<cdiv(tot, 256), 256, 0, st>>>(in, N, C, H, W, Cp, (float*)out);
}

// ---------------------------------------------------------------- FaceNet head
// AdaptiveAvgPool2d(1) -> Linear 1792->512 (no bias) -> BatchNorm1d -> F.normalize
// (facenet.py:144-147,153); weights fp32 [512][1792].  Pool, FC + BN on the fp32 GEMM, normalise.
template <typename T>
__global__ __launch_bounds__(256) void k_facenet_pool(const T* __restrict__ x, int N, int HW, int C,
                                                      float* __restrict__ pooled) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= (int64_t)N * C) return;
    const int c = (int)(i % C);
    const int64_t n = i / C;
    int side = 1;
    while (side * side < HW) side++;
    const T* xn = x + n * HW * C;
    float s = 0.f;
    for (int k = 0; k < HW; k++) s = s + to_f(xn[(int64_t)k * C + c]);
    pooled[i] = __fdiv_rn(__fdiv_rn(s, (float)side), (float)side);
}

// F.normalize(p=2, dim=1): one wave per embedding
__global__ __launch_bounds__(64) void k_l2_normalize(const float* __restrict__ y, int D, float* __restrict__ out) {
    const int64_t n = blockIdx.x;
    const int lane = threadIdx.x;
    float sq = 0.f;
    for (int d = lane; d < D; d += 64) {
        const float v = y[n * D + d];
        sq = fmaf(v, v, sq);
    }
    for (int off = 32; off > 0; off >>= 1) sq += __shfl_xor(sq, off);
    const float nrm = fmaxf(sqrtf(sq), 1e-12f);
    for (int d = lane; d < D; d += 64) out[n * D + d] = __fdiv_rn(y[n * D + d], nrm);
}

void launch_facenet_head(const void* x, int N, int HW, int C, const float* w, const float* alpha, const float* beta,
                         int D, float* out, float* scratch, bool bf16, hipStream_t st) {
    if (N <= 0) return;
    float* pooled = scratch;                 // [N][C]
    float* y = scratch + (size_t)N * C;      // [N][D] before the L2 normalisation
    const int64_t nc = (int64_t)N * C;
    if (bf16)
        k_facenet_pool<__bf16><<<cdiv(nc, 256), 256, 0, st>>>((const __bf16*)x, N, HW, C, pooled);
    else
        k_facenet_pool<float><<<cdiv(nc, 256), 256, 0, st>>>((const float*)x, N, HW, C, pooled);
    // last_linear + last_bn: a 1x1 "conv" over the pooled rows on the fp32 MFMA GEMM (split-K
    // over the 1792-deep K for a full grid), BN folded into the epilogue
    ConvParams p{};
    p.in = pooled;
    p.w = w;
    p.out = y;
    p.alpha = alpha;
    p.beta = beta;
    p.scale = 1.f;
    p.N = N;
    p.H = p.W = p.OH = p.OW = 1;
    p.Cin = C;
    p.KH = p.KW = p.sh = p.sw = 1;
    p.Cout = D;
    p.K = C;
    p.M = N;
    p.out_cstride = D;
    p.split_fp32 = 1;
    launch_conv(p, false, st);
    k_l2_normalize<<<N, 64, 0, st>>>(y, D, out);
}

}  // namespace vtf

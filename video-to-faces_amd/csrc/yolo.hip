// YOLOv3 face detector (src/videotofaces/detectors/yolo.py:17-191) on gfx950.
//
//   letterbox  k_letterbox: cv2 INTER_LINEAR keep-ratio resize + BGR->RGB + /255 + zero pad
//              to a multiple of 32 (prep.py:12-92), one pass from the uint8 frames in HBM to
//              the NHWC (C padded to 8) network input.
//   net        72 ConvUnits (Conv -> BN -> LeakyReLU(0.1), yolo.py:17-18) + 3 pred convs, each
//              one launch of the implicit-GEMM MFMA kernel (conv.hip) with BN/LeakyReLU and
//              the Darknet residual (y + x after the activation, yolo.py:28-31) fused in the
//              epilogue.  Concats are channel slices: the stage-3/4 backbone outputs are
//              written straight into the neck's concat buffers, and the neck's 1x1 laterals
//              write their nearest x2 upsample (yolo.py:87,91) into the other slice from the
//              epilogue -- no interpolate / cat kernels.
//   decode     k_yolo_flag + scan + k_yolo_emit: sigmoid gates obj >= 0.005, cls > 0.05,
//              score = cls * obj, yolo box decode (bbox.py:17-27) against the implicit
//              centre priors (anchor.py:20-64) -- compaction keeps the reference's
//              (image, prior) order.
//   nms        nms_multi: one torchvision batched_nms(0.45) call per image (post.py:4-10),
//              then top-100 and scale_boxes (bbox.py:63-67) in k_yolo_final.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "blob.hpp"
#include "boxes.hpp"
#include "common.hpp"
#include "conv.hpp"
#include "conv_dev.hpp"
#include "nms.hpp"

namespace vtf {

struct YUnit {
    int cin, cout, k, s, cin_pad;
    int cout_p;    // bf16x3 mode: Cout padded to 8 (the pred convs' 18 -> 24; zero weight rows)
    void* w;       // [cout][k][k][cin_pad], element = precision
    float* alpha;  // folded BN (ConvUnit)
    float* beta;
    float* bias;   // pred conv bias (no BN, no activation)
};

struct Yolo {
    int device = 0;
    bool bf16 = false;
    // bf16x3 (fp32-grade products on the bf16 matrix cores, conv_dma MODE 2): activations and
    // weights in the split-triple layout (6 bytes per element), pred-conv maps fp32
    bool x3 = false;
    size_t es() const { return x3 ? 6 : (bf16 ? 2 : 4); }
    hipStream_t st = 0;
    std::vector<YUnit> U;
    std::vector<void*> allocs;
    Arena ar;
    bool prof = false;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double prof_ms = 0, prof_flops = 0;
    int64_t prof_launches = 0, prof_frames = 0;
    double flops = 0;
    int64_t launches = 0;
    ~Yolo() {
        for (void* p : allocs) (void)hipFree(p);
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
    }
    template <class T>
    T* upload(const std::vector<T>& v) {
        void* p = nullptr;
        VTF_HIP(hipMalloc(&p, v.size() * sizeof(T) + 16));
        VTF_HIP(hipMemcpy(p, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
        allocs.push_back(p);
        return (T*)p;
    }
};

struct YG {
    int cin, cout, k, s, pred;
};

// every conv in reference state_dict order (videotofaces/specs.py yolo_spec)
static std::vector<YG> yolo_geometry() {
    std::vector<YG> g = {{3, 32, 3, 1, 0}};  // Darknet53.conv1 (yolo.py:38)
    const int L[5] = {1, 2, 8, 8, 4}, C[5] = {64, 128, 256, 512, 1024};
    for (int i = 0; i < 5; i++) {
        g.push_back({C[i] / 2, C[i], 3, 2, 0});
        for (int j = 0; j < L[i]; j++) {
            g.push_back({C[i], C[i] / 2, 1, 1, 0});
            g.push_back({C[i] / 2, C[i], 3, 1, 0});
        }
    }
    auto det = [&](int cin, int c) {  // DetectionBlock (yolo.py:57-70)
        g.push_back({cin, c, 1, 1, 0});
        g.push_back({c, 2 * c, 3, 1, 0});
        g.push_back({2 * c, c, 1, 1, 0});
        g.push_back({c, 2 * c, 3, 1, 0});
        g.push_back({2 * c, c, 1, 1, 0});
    };
    det(1024, 512);
    g.push_back({512, 256, 1, 1, 0});
    det(768, 256);
    g.push_back({256, 128, 1, 1, 0});
    det(384, 128);
    g.push_back({512, 1024, 3, 1, 0});  // convs_bridge (yolo.py:100-104)
    g.push_back({256, 512, 3, 1, 0});
    g.push_back({128, 256, 3, 1, 0});
    g.push_back({1024, 18, 1, 1, 1});  // convs_pred (yolo.py:106-111)
    g.push_back({512, 18, 1, 1, 1});
    g.push_back({256, 18, 1, 1, 1});
    return g;
}
constexpr int Y_UNITS = 75, Y_BRIDGE = 69, Y_PRED = 72;

static void build(Yolo& Y, const float* params, int64_t n_params) {
    std::vector<YG> geo = yolo_geometry();
    VTF_CHECK((int)geo.size() == Y_UNITS, VTF_E_ARG, "yolo: geometry");
    int64_t src = 0;
    auto take = [&](int64_t n) {
        VTF_CHECK(src + n <= n_params, VTF_E_ARG, "yolo: parameter buffer too small");
        const float* p = params + src;
        src += n;
        return p;
    };
    for (const YG& g : geo) {
        YUnit u{};
        u.cin = g.cin;
        u.cout = g.cout;
        u.k = g.k;
        u.s = g.s;
        u.cin_pad = (g.cin + 7) / 8 * 8;
        const float* w = take((int64_t)g.cout * g.cin * g.k * g.k);
        int K = g.k * g.k * u.cin_pad;
        std::vector<float> wt((size_t)g.cout * K, 0.f);
        for (int co = 0; co < g.cout; co++)
            for (int ci = 0; ci < g.cin; ci++)
                for (int y = 0; y < g.k; y++)
                    for (int x = 0; x < g.k; x++)
                        wt[(size_t)co * K + (y * g.k + x) * u.cin_pad + ci] =
                            w[(((size_t)co * g.cin + ci) * g.k + y) * g.k + x];
        u.cout_p = g.cout;
        if (Y.x3) {
            // split-triple rows [cout_p][K/8][b0 x 8 | b1 x 8 | b2 x 8] (conv_dev.hpp), zero rows past Cout
            u.cout_p = (g.cout + 7) / 8 * 8;
            std::vector<uint16_t> w3((size_t)u.cout_p * K * 3, 0);
            for (int co = 0; co < g.cout; co++)
                for (int k = 0; k < K; k++) {
                    const float v = wt[(size_t)co * K + k];
                    const uint16_t b0 = f2bf(v);
                    const float r1 = v - __builtin_bit_cast(float, (uint32_t)b0 << 16);
                    const uint16_t b1 = f2bf(r1);
                    const uint16_t b2 = f2bf(r1 - __builtin_bit_cast(float, (uint32_t)b1 << 16));
                    uint16_t* c = &w3[((size_t)co * (K / 8) + k / 8) * 24 + (k & 7)];
                    c[0] = b0;
                    c[8] = b1;
                    c[16] = b2;
                }
            u.w = Y.upload(w3);
        } else if (Y.bf16) {
            std::vector<uint16_t> wb(wt.size());
            for (size_t i = 0; i < wt.size(); i++) wb[i] = f2bf(wt[i]);
            u.w = Y.upload(wb);
        } else {
            u.w = Y.upload(wt);
        }
        if (g.pred) {
            const float* b = take(g.cout);
            std::vector<float> bv(b, b + g.cout);
            bv.resize(u.cout_p, 0.f);
            u.bias = Y.upload(bv);
        } else {
            // BatchNorm2d(eps 1e-5) folded the way torch's CPU inference kernel does it
            // (invstd = 1/sqrt(var+eps), alpha = invstd*w, beta = b - mean*alpha)
            const float* bw = take(g.cout);
            const float* bb = take(g.cout);
            const float* bm = take(g.cout);
            const float* bv = take(g.cout);
            std::vector<float> a(g.cout), be(g.cout);
            for (int c = 0; c < g.cout; c++) {
                float invstd = 1.f / std::sqrt(bv[c] + 1e-5f);
                a[c] = invstd * bw[c];
                be[c] = bb[c] - bm[c] * a[c];
            }
            u.alpha = Y.upload(a);
            u.beta = Y.upload(be);
        }
        Y.U.push_back(u);
    }
    VTF_CHECK(src == n_params, VTF_E_ARG, "yolo: expected 61,576,342 parameters");
}

// ------------------------------------------------------------------ letterbox
// keep-ratio size exactly as resize_cv2 computes it in Python doubles (prep.py:71-73)
static void used_size(int H, int W, int& h, int& w) {
    double scl = std::min(608.0 / std::min(H, W), 608.0 / std::max(H, W));
    h = (int)(H * scl + 0.5);
    w = (int)(W * scl + 0.5);
}

template <typename T>
__global__ void k_letterbox(const uint8_t* __restrict__ frames, int64_t fstride, int64_t rstride, int H, int W, int h,
                            int w, int Hp, int Wp, int64_t total, T* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    int dx = (int)(i % Wp);
    int dy = (int)((i / Wp) % Hp);
    int64_t b = i / ((int64_t)Wp * Hp);
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (dy < h && dx < w) {
        const uint8_t* base = frames + b * fstride;
        int u[3];
        if (h == H && w == W) {
            const uint8_t* p = base + (int64_t)dy * rstride + dx * 3;
            u[0] = p[0];
            u[1] = p[1];
            u[2] = p[2];
        } else {
            int sx0, sx1, a0, a1, sy0, sy1, b0, b1;
            bool ex, ey;
            lin_coef(dx, W, w, sx0, sx1, a0, a1, ex);
            lin_coef(dy, H, h, sy0, sy1, b0, b1, ey);
            (void)ey;
            const uint8_t* r0 = base + (int64_t)sy0 * rstride;
            const uint8_t* r1 = base + (int64_t)sy1 * rstride;
#pragma unroll
            for (int ch = 0; ch < 3; ch++) {
                int h0 = ex ? r0[sx0 * 3 + ch] * 2048 : r0[sx0 * 3 + ch] * a0 + r0[sx1 * 3 + ch] * a1;
                int h1 = ex ? r1[sx0 * 3 + ch] * 2048 : r1[sx0 * 3 + ch] * a0 + r1[sx1 * 3 + ch] * a1;
                int t = ((((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16) + 2) >> 2;
                u[ch] = min(255, max(0, t));
            }
        }
        // to_tensors(means=None, stdvs=255, to_rgb=True): t[:, :, [2,1,0]] / 255 (prep.py:27-48)
        for (int oc = 0; oc < 3; oc++) v[oc] = __fdiv_rn((float)u[2 - oc], 255.f);
    }
    T* o = out + i * 8;
#pragma unroll
    for (int c = 0; c < 8; c++) o[c] = (T)v[c];
}

// the same pass writing the split-triple layout (8 channels = one 48-byte chunk per pixel)
__global__ void k_letterbox_s3(const uint8_t* __restrict__ frames, int64_t fstride, int64_t rstride, int H, int W,
                               int h, int w, int Hp, int Wp, int64_t total, char* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    int dx = (int)(i % Wp);
    int dy = (int)((i / Wp) % Hp);
    int64_t b = i / ((int64_t)Wp * Hp);
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (dy < h && dx < w) {
        const uint8_t* base = frames + b * fstride;
        int u[3];
        if (h == H && w == W) {
            const uint8_t* p = base + (int64_t)dy * rstride + dx * 3;
            u[0] = p[0];
            u[1] = p[1];
            u[2] = p[2];
        } else {
            int sx0, sx1, a0, a1, sy0, sy1, b0, b1;
            bool ex, ey;
            lin_coef(dx, W, w, sx0, sx1, a0, a1, ex);
            lin_coef(dy, H, h, sy0, sy1, b0, b1, ey);
            (void)ey;
            const uint8_t* r0 = base + (int64_t)sy0 * rstride;
            const uint8_t* r1 = base + (int64_t)sy1 * rstride;
#pragma unroll
            for (int ch = 0; ch < 3; ch++) {
                int h0 = ex ? r0[sx0 * 3 + ch] * 2048 : r0[sx0 * 3 + ch] * a0 + r0[sx1 * 3 + ch] * a1;
                int h1 = ex ? r1[sx0 * 3 + ch] * 2048 : r1[sx0 * 3 + ch] * a0 + r1[sx1 * 3 + ch] * a1;
                int t = ((((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16) + 2) >> 2;
                u[ch] = min(255, max(0, t));
            }
        }
        for (int oc = 0; oc < 3; oc++) v[oc] = __fdiv_rn((float)u[2 - oc], 255.f);
    }
    s3_store8(out + i * 48, v);
}

// ------------------------------------------------------------------ stem head (bf16x3)
// The letterbox (k_letterbox_s3's arithmetic: OpenCV INTER_LINEAR restated, / 255, the S3 split)
// straight into Darknet's first conv (3x3, stride 1, pad 1, 3 -> 32, BN + LeakyReLU(0.1)):
// a tile of 8 x 16 canvas pixels computes its 10 x 18 letterboxed input patch into LDS (48-byte
// S3 pixels: a 16-lane group reads 16 consecutive pixels over all 64 banks) and runs the conv from
// there with k_conv_dma3's MFMA chains (the same k-steps, lane -> k map, six products per step in
// the same order, acc + accx, the same epilogue and S3 stores): bit-identical to letterbox ->
// k_conv_dma3, without the canvas (329 MB per 32 720p frames) going through HBM and with the
// conv's small tiles at many workgroups per CU instead of 73 KB of DMA stages.
constexpr int YS_TH = 8, YS_TW = 16, YS_PH = YS_TH + 2, YS_PW = YS_TW + 2, YS_COUT = 32;
typedef __attribute__((ext_vector_type(4))) float f4;

struct YStemP {
    const uint8_t* frames;
    int64_t fstride, rstride;
    int H, W, h, w, Hp, Wp, tiles_x, tiles_per_img;
    const char* w3;  // conv weights, S3 [32][9 chunks][48 B] (k = tap * 8 + c)
    const float *al, *be;
    char* out;       // S3 [B][Hp][Wp][32]
};

__global__ __launch_bounds__(256) void k_yolo_stem(YStemP p) {
    __shared__ __attribute__((aligned(16))) char P[YS_PH * YS_PW * 48];
    __shared__ __attribute__((aligned(16))) float E[YS_TH * YS_TW * (YS_COUT + 4)];
    __shared__ int4 ycf[YS_PH], xcf[YS_PW];  // lin_coef (s0, s1, c0, c1); x: the edge flag in s1's sign
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int b = blockIdx.x / p.tiles_per_img, t = blockIdx.x - b * p.tiles_per_img;
    const int ty = t / p.tiles_x, oy0 = ty * YS_TH, ox0 = (t - ty * p.tiles_x) * YS_TW;
    const bool direct = p.h == p.H && p.w == p.W;
    if (!direct) {
        if (tid < YS_PH) {
            const int dy = min(max(oy0 - 1 + tid, 0), p.h - 1);
            int s0, s1, c0, c1;
            bool e;
            lin_coef(dy, p.H, p.h, s0, s1, c0, c1, e);
            ycf[tid] = make_int4(s0, s1, c0, c1);
        } else if (tid >= 64 && tid < 64 + YS_PW) {
            const int dx = min(max(ox0 - 1 + tid - 64, 0), p.w - 1);
            int s0, s1, c0, c1;
            bool e;
            lin_coef(dx, p.W, p.w, s0, s1, c0, c1, e);
            xcf[tid - 64] = make_int4(s0, e ? -1 - s1 : s1, c0, c1);
        }
    }
    __syncthreads();
    const uint8_t* base = p.frames + (int64_t)b * p.fstride;
    for (int e = tid; e < YS_PH * YS_PW; e += 256) {
        const int r = e / YS_PW, c = e - r * YS_PW;
        const int dy = oy0 - 1 + r, dx = ox0 - 1 + c;
        float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (dy >= 0 && dx >= 0 && dy < p.h && dx < p.w) {
            int u[3];
            if (direct) {
                const uint8_t* q = base + (int64_t)dy * p.rstride + dx * 3;
                u[0] = q[0], u[1] = q[1], u[2] = q[2];
            } else {
                const int4 yc = ycf[r], xc = xcf[c];
                const bool ex = xc.y < 0;
                const int sx1 = ex ? -1 - xc.y : xc.y;
                const uint8_t* r0 = base + (int64_t)yc.x * p.rstride;
                const uint8_t* r1 = base + (int64_t)yc.y * p.rstride;
#pragma unroll
                for (int ch = 0; ch < 3; ch++) u[ch] = blob_lin(r0, r1, xc.x, sx1, xc.z, xc.w, ex, yc.z, yc.w, ch);
            }
            for (int oc = 0; oc < 3; oc++) v[oc] = __fdiv_rn((float)u[2 - oc], 255.f);
        }
        s3_store8(P + e * 48, v);
    }
    // B (weights): lane (channel 16 j + (lane & 15), chunk 4 s + (lane >> 4)), three planes
    const int g = lane >> 4, n16 = lane & 15;
    f4 acc[2][2], accx[2][2];
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) acc[i][j] = accx[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    __syncthreads();
#pragma unroll
    for (int s = 0; s < 3; s++) {
        const int tap = 4 * s + g, ky = tap / 3, kx = tap - 3 * ky;
        bf16x8 bw[2][3];
#pragma unroll
        for (int j = 0; j < 2; j++)
#pragma unroll
            for (int pl = 0; pl < 3; pl++)
                bw[j][pl] = tap < 9 ? *(const bf16x8*)(p.w3 + ((16 * j + n16) * 9 + tap) * 48 + 16 * pl) : bf16x8{};
#pragma unroll
        for (int i = 0; i < 2; i++) {
            // fragment i of this wave: tile row 2 wave + i, pixel n16 of it
            bf16x8 a[3];
            const char* q = P + ((2 * wave + i + ky) * YS_PW + n16 + kx) * 48;
#pragma unroll
            for (int pl = 0; pl < 3; pl++) a[pl] = tap < 9 ? *(const bf16x8*)(q + 16 * pl) : bf16x8{};
#pragma unroll
            for (int j = 0; j < 2; j++) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bw[j][0], acc[i][j], 0, 0, 0);
                accx[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bw[j][1], accx[i][j], 0, 0, 0);
                accx[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], bw[j][0], accx[i][j], 0, 0, 0);
                accx[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], bw[j][2], accx[i][j], 0, 0, 0);
                accx[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], bw[j][1], accx[i][j], 0, 0, 0);
                accx[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], bw[j][0], accx[i][j], 0, 0, 0);
            }
        }
    }
    constexpr int LDE = YS_COUT + 4;
#pragma unroll
    for (int i = 0; i < 2; i++)
#pragma unroll
        for (int j = 0; j < 2; j++) {
            const f4 v = acc[i][j] + accx[i][j];
#pragma unroll
            for (int q = 0; q < 4; q++) E[(16 * (2 * wave + i) + 4 * g + q) * LDE + 16 * j + n16] = v[q];
        }
    __syncthreads();
    // conv_epilogue8 (BN fmaf, LeakyReLU(0.1)) and the S3 store of 8 channels per item
    for (int it = tid; it < YS_TH * YS_TW * (YS_COUT / 8); it += 256) {
        const int m = it >> 2, c8 = it & 3;
        const int oy = oy0 + (m >> 4), ox = ox0 + (m & 15);
        float v[8];
#pragma unroll
        for (int e = 0; e < 8; e++) {
            float x = E[m * LDE + 8 * c8 + e];
            x = fmaf(x, p.al[8 * c8 + e], p.be[8 * c8 + e]);
            x = x > 0.f ? x : x * 0.1f;
            v[e] = x;
        }
        const int64_t gm = ((int64_t)b * p.Hp + oy) * p.Wp + ox;
        s3_store8(p.out + (gm * YS_COUT + 8 * c8) / 8 * 48, v);
    }
}

// NCHW fp32 (C <= 8) -> split-triple NHWC with 8 channels (vtf_yolo_net's input)
__global__ void k_nchw_to_s3(const float* __restrict__ in, int64_t N, int C, int H, int W, char* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N * H * W) return;
    const int64_t n = i / ((int64_t)H * W), hw = i % ((int64_t)H * W);
    float v[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    for (int c = 0; c < C; c++) v[c] = in[(n * C + c) * H * W + hw];
    s3_store8(out + i * 48, v);
}

// first 18 channels of the padded (24-channel) fp32 pred-conv output
__global__ void k_compact18(const float* __restrict__ in, int64_t rows, float* __restrict__ out) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= rows * 18) return;
    out[i] = in[(i / 18) * 24 + i % 18];
}

static void launch_letterbox(const uint8_t* frames, int64_t fstride, int64_t rstride, int B, int H, int W, int h, int w,
                             int Hp, int Wp, bool bf16, void* out, hipStream_t st, bool x3 = false) {
    int64_t total = (int64_t)B * Hp * Wp;
    if (x3)
        k_letterbox_s3<<<cdiv(total, 256), 256, 0, st>>>(frames, fstride, rstride, H, W, h, w, Hp, Wp, total, (char*)out);
    else if (bf16)
        k_letterbox<__bf16><<<cdiv(total, 256), 256, 0, st>>>(frames, fstride, rstride, H, W, h, w, Hp, Wp, total,
                                                               (__bf16*)out);
    else
        k_letterbox<float><<<cdiv(total, 256), 256, 0, st>>>(frames, fstride, rstride, H, W, h, w, Hp, Wp, total,
                                                              (float*)out);
}

// ------------------------------------------------------------------ net
static void unit(Yolo& Y, int li, const void* in, int in_cs, int N, int H, int W, void* out, int out_cs, int out_coff,
                 const void* res = nullptr, int res_cs = 0, bool up2 = false) {
    const YUnit& u = Y.U[li];
    ConvParams p{};
    p.in = in;
    p.w = u.w;
    p.out = out;
    p.N = N;
    p.H = H;
    p.W = W;
    p.Cin = u.cin_pad;
    p.in_cstride = in_cs == u.cin_pad ? 0 : in_cs;
    p.KH = p.KW = u.k;
    p.sh = p.sw = u.s;
    p.ph = p.pw = (u.k - 1) / 2;
    p.OH = (H + 2 * p.ph - u.k) / u.s + 1;
    p.OW = (W + 2 * p.pw - u.k) / u.s + 1;
    p.Cout = u.cout;
    p.K = u.k * u.k * u.cin_pad;
    p.M = (int64_t)N * p.OH * p.OW;
    p.out_cstride = out_cs;
    p.out_coff = out_coff;
    p.scale = 1.f;
    if (u.bias) {
        p.bias = u.bias;
        p.out_f32 = 1;
    } else {
        p.alpha = u.alpha;
        p.beta = u.beta;
        p.leaky = 1;
        p.slope = 0.1f;  // LeakyReLU(0.1) -> (float)0.1
    }
    if (res) {
        p.res = res;
        p.res_cstride = res_cs;
        p.res_post = 1;
    }
    p.up2 = up2 ? 1 : 0;
    if (Y.x3) {
        // split-triple operands on the bf16 matrix cores; the pred convs write their padded
        // 24-channel fp32 maps to scratch, compacted to the 18-channel layout the decode reads
        p.s3 = 1;
        p.split_fp32 = 1;  // tail tiles may be split along K (slice-order reduction; parity is a tolerance)
        p.Cout = u.cout_p;
        if (u.bias) {
            float* tmp = Y.ar.get<float>(89, (size_t)p.M * u.cout_p);
            p.out = tmp;
            p.out_cstride = u.cout_p;
            launch_conv_dma(p, false, Y.st);
            k_compact18<<<cdiv(p.M * 18, 256), 256, 0, Y.st>>>(tmp, p.M, (float*)out);
        } else {
            launch_conv_dma(p, false, Y.st);
        }
    } else {
        launch_conv(p, Y.bf16, Y.st);
    }
    Y.flops += 2.0 * (double)p.M * u.cout * u.k * u.k * u.cin;
    Y.launches++;
}

// the frames a fused stem head letterboxes itself (bf16x3 mode)
struct YStemIn {
    const uint8_t* frames;
    int64_t fstride, rstride;
    int H, W, h, w;
};

// bf16x3 stem head on by default (VTF_YOLO_STEM=0: letterbox + the first conv's launch)
static bool stem_on() {
    const char* e = std::getenv("VTF_YOLO_STEM");  // (read per call: tests switch it in-process)
    return !(e && std::atoi(e) == 0);
}

// x0: NHWC [B,Hp,Wp,8] -> maps NHWC fp32 [B,Hp/32,Wp/32,18], [.., /16, ..], [.., /8, ..]; or
// (stem, bf16x3 mode) the frames, letterboxed inside the first conv's launch
static void net(Yolo& Y, const void* x0, int B, int Hp, int Wp, float* maps[3], const YStemIn* stem = nullptr) {
    VTF_CHECK(Hp % 32 == 0 && Wp % 32 == 0 && Hp > 0 && Wp > 0, VTF_E_ARG, "yolo: input must be padded to x32");
    const size_t es = Y.es();
    const size_t full = (size_t)B * Hp * Wp * 32;
    char* A = (char*)Y.ar.get(80, full * es);
    char* Bf = (char*)Y.ar.get(81, full * es);
    char* T = (char*)Y.ar.get(82, full / 4 * es);
    const int H3 = Hp / 8, W3 = Wp / 8, H4 = Hp / 16, W4 = Wp / 16, H5 = Hp / 32, W5 = Wp / 32;
    char* C3 = (char*)Y.ar.get(83, (size_t)B * H3 * W3 * 384 * es);
    char* C2 = (char*)Y.ar.get(84, (size_t)B * H4 * W4 * 768 * es);
    char* X5 = (char*)Y.ar.get(85, (size_t)B * H5 * W5 * 1024 * es);
    char* Y3 = (char*)Y.ar.get(86, (size_t)B * H5 * W5 * 512 * es);
    char* Y2 = (char*)Y.ar.get(87, (size_t)B * H4 * W4 * 256 * es);
    char* Y1 = (char*)Y.ar.get(88, (size_t)B * H3 * W3 * 128 * es);
    Y.flops = 0;
    Y.launches = 0;
    if (Y.prof) VTF_HIP(hipEventRecord(Y.ev0, Y.st));
    int li = 0;
    // Darknet53 (yolo.py:34-54)
    if (stem) {
        const YUnit& u = Y.U[0];
        VTF_CHECK(Y.x3 && u.k == 3 && u.s == 1 && u.cin_pad == 8 && u.cout_p == 32 && !u.bias, VTF_E_ARG,
                  "yolo: stem head shape");
        YStemP sp;
        sp.frames = stem->frames;
        sp.fstride = stem->fstride;
        sp.rstride = stem->rstride;
        sp.H = stem->H;
        sp.W = stem->W;
        sp.h = stem->h;
        sp.w = stem->w;
        sp.Hp = Hp;
        sp.Wp = Wp;
        sp.tiles_x = Wp / YS_TW;
        sp.tiles_per_img = sp.tiles_x * (Hp / YS_TH);
        sp.w3 = (const char*)u.w;
        sp.al = u.alpha;
        sp.be = u.beta;
        sp.out = A;
        k_yolo_stem<<<(unsigned)((int64_t)B * sp.tiles_per_img), 256, 0, Y.st>>>(sp);
        Y.flops += 2.0 * (double)B * Hp * Wp * u.cout * 9 * u.cin;
        Y.launches++;
        li++;
    } else {
        unit(Y, li++, x0, 8, B, Hp, Wp, A, 32, 0);
    }
    char* cur = A;
    int cur_cs = 32, H = Hp, W = Wp;
    const int L[5] = {1, 2, 8, 8, 4}, C[5] = {64, 128, 256, 512, 1024};
    for (int i = 0; i < 5; i++) {
        char* dst;
        int dcs, doff;
        if (i == 2) {
            dst = C3, dcs = 384, doff = 128;  // x3 -> cat((t, x1)) slice (yolo.py:92)
        } else if (i == 3) {
            dst = C2, dcs = 768, doff = 256;  // x4 -> cat((t, x2)) slice (yolo.py:88)
        } else if (i == 4) {
            dst = X5, dcs = 1024, doff = 0;
        } else {
            dst = cur == A ? Bf : A, dcs = C[i], doff = 0;
        }
        unit(Y, li++, cur, cur_cs, B, H, W, dst, dcs, doff);
        H = (H - 1) / 2 + 1;
        W = (W - 1) / 2 + 1;
        char* x = dst + (size_t)doff * es;
        for (int j = 0; j < L[i]; j++) {  // ResBlock: y = conv2(conv1(x)); x = y + x (yolo.py:21-31)
            unit(Y, li++, x, dcs, B, H, W, T, C[i] / 2, 0);
            unit(Y, li++, T, C[i] / 2, B, H, W, dst, dcs, doff, x, dcs);
        }
        cur = x;
        cur_cs = dcs;
    }
    // neck (yolo.py:73-94)
    auto det = [&](const void* in, int in_cs, int h, int w, int c, char* out) {
        unit(Y, li++, in, in_cs, B, h, w, A, c, 0);
        unit(Y, li++, A, c, B, h, w, Bf, 2 * c, 0);
        unit(Y, li++, Bf, 2 * c, B, h, w, A, c, 0);
        unit(Y, li++, A, c, B, h, w, Bf, 2 * c, 0);
        unit(Y, li++, Bf, 2 * c, B, h, w, out, c, 0);
    };
    det(X5, 1024, H5, W5, 512, Y3);
    unit(Y, li++, Y3, 512, B, H5, W5, C2, 768, 0, nullptr, 0, true);
    det(C2, 768, H4, W4, 256, Y2);
    unit(Y, li++, Y2, 256, B, H4, W4, C3, 384, 0, nullptr, 0, true);
    det(C3, 384, H3, W3, 128, Y1);
    VTF_CHECK(li == Y_BRIDGE, VTF_E_ARG, "yolo: layer walk mismatch");
    // head (yolo.py:114-120)
    const char* ys[3] = {Y3, Y2, Y1};
    const int hs[3] = {H5, H4, H3}, ws[3] = {W5, W4, W3}, cs[3] = {512, 256, 128};
    for (int i = 0; i < 3; i++) {
        unit(Y, Y_BRIDGE + i, ys[i], cs[i], B, hs[i], ws[i], A, 2 * cs[i], 0);
        unit(Y, Y_PRED + i, A, 2 * cs[i], B, hs[i], ws[i], maps[i], 18, 0);
    }
    if (Y.prof) {
        VTF_HIP(hipEventRecord(Y.ev1, Y.st));
        VTF_HIP(hipEventSynchronize(Y.ev1));
        float ms = 0;
        VTF_HIP(hipEventElapsedTime(&ms, Y.ev0, Y.ev1));
        Y.prof_ms += ms;
        Y.prof_flops += Y.flops;
        Y.prof_launches += Y.launches;
        Y.prof_frames += B;
    }
}

// ------------------------------------------------------------------ decode + NMS
struct YLevel {
    const float* map;  // NHWC [B,h,w,18]
    int h, w, stride;
    int64_t off;       // first prior of the level within an image
    float aw[3], ah[3];
};
struct YDec {
    YLevel L[3];
    int64_t dim;  // priors per image (13,167 at 352x608)
};

// YOLOv3.bases (yolo.py:125-129)
static YDec make_dec(float* const maps[3], int Hp, int Wp) {
    static const int strides[3] = {32, 16, 8};
    static const float anc[3][3][2] = {{{116, 90}, {156, 198}, {373, 326}},
                                       {{30, 61}, {62, 45}, {59, 119}},
                                       {{10, 13}, {16, 30}, {33, 23}}};
    YDec d{};
    int64_t off = 0;
    for (int l = 0; l < 3; l++) {
        YLevel& L = d.L[l];
        L.map = maps[l];
        L.stride = strides[l];
        L.h = (Hp + strides[l] - 1) / strides[l];
        L.w = (Wp + strides[l] - 1) / strides[l];
        L.off = off;
        for (int a = 0; a < 3; a++) {
            L.aw[a] = anc[l][a][0];
            L.ah[a] = anc[l][a][1];
        }
        off += (int64_t)L.h * L.w * 3;
    }
    d.dim = off;
    return d;
}

__device__ inline float sigm(float x) { return 1.f / (1.f + expf(-x)); }

__device__ inline const float* prior_row(const YDec& d, int64_t b, int64_t p, int& l, int& a, int& x, int& y) {
    l = p < d.L[1].off ? 0 : (p < d.L[2].off ? 1 : 2);
    const YLevel& L = d.L[l];
    int64_t q = p - L.off;
    a = (int)(q % 3);
    int64_t cell = q / 3;
    x = (int)(cell % L.w);
    y = (int)(cell / L.w);
    return L.map + ((b * L.h * L.w + cell) * 18 + a * 6);
}

// obj = sigmoid(t4) >= 0.005, then cls = sigmoid(t5) > 0.05 (yolo.py:156-166)
__global__ void k_yolo_flag(YDec d, int64_t total, int32_t* __restrict__ flag) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    int l, a, x, y;
    const float* t = prior_row(d, i / d.dim, i % d.dim, l, a, x, y);
    float obj = sigm(t[4]);
    float cls = sigm(t[5]);
    flag[i] = (obj >= 0.005f && cls > 0.05f) ? 1 : 0;
}

// decode_boxes(mode='yolo') (bbox.py:24-26) for the surviving priors, at their compacted slot
__global__ void k_yolo_emit(YDec d, int64_t total, const int32_t* __restrict__ flag, const int32_t* __restrict__ incl,
                            float4* __restrict__ boxes, float* __restrict__ score, int32_t* __restrict__ call,
                            int32_t* __restrict__ cls) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total || !flag[i]) return;
    int64_t b = i / d.dim;
    int l, a, x, y;
    const float* t = prior_row(d, b, i % d.dim, l, a, x, y);
    const YLevel& L = d.L[l];
    float s = (float)L.stride;
    // get_priors(loc='center'): arange * stride + stride / 2 (anchor.py:54-58)
    float cx = (float)x * s + s * 0.5f;
    float cy = (float)y * s + s * 0.5f;
    float px = s * (sigm(t[0]) - 0.5f) + cx;
    float py = s * (sigm(t[1]) - 0.5f) + cy;
    float pw = L.aw[a] * expf(t[2]);
    float ph = L.ah[a] * expf(t[3]);
    float hw = pw / 2.f, hh = ph / 2.f;
    int32_t o = incl[i] - 1;
    boxes[o] = make_float4(px - hw, py - hh, px + hw, py + hh);
    score[o] = sigm(t[5]) * sigm(t[4]);
    call[o] = (int32_t)b;
    cls[o] = 0;
}

__global__ void k_yolo_counts(const int32_t* __restrict__ incl, int64_t dim, int B, int32_t* __restrict__ out) {
    int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= B) return;
    int32_t hi = incl[(int64_t)(b + 1) * dim - 1];
    int32_t lo = b ? incl[(int64_t)b * dim - 1] : 0;
    out[b] = hi - lo;
}

// keep[:100] per image, then boxes * (W/w, H/h, W/w, H/h) (post.py:8, bbox.py:63-67)
__global__ void k_yolo_final(const int32_t* __restrict__ keep, const int64_t* __restrict__ offs, const float4* boxes,
                             const float* score, float sx, float sy, int top, float* __restrict__ out) {
    int b = blockIdx.x;
    int64_t kb = offs[3 * b], nb = offs[3 * b + 1], ob = offs[3 * b + 2];
    for (int t = threadIdx.x; t < nb && t < top; t += blockDim.x) {
        int32_t e = keep[kb + t];
        float4 v = boxes[e];
        float* o = out + (ob + t) * 5;
        o[0] = v.x * sx;
        o[1] = v.y * sy;
        o[2] = v.z * sx;
        o[3] = v.w * sy;
        o[4] = score[e];
    }
}

struct YOut {
    std::vector<float> rows;  // [n,5] x1,y1,x2,y2,score (host copy, when requested)
    std::vector<int32_t> counts;
    const float* d_rows = nullptr;  // the same rows in HBM
    int64_t n = 0;
    bool host = true;
};

static void postprocess(Yolo& Y, float* const maps[3], int B, int Hp, int Wp, int H, int W, YOut& out) {
    hipStream_t st = Y.st;
    YDec d = make_dec(maps, Hp, Wp);
    int64_t total = (int64_t)B * d.dim;
    VTF_CHECK(total < ((int64_t)1 << 31), VTF_E_LIMIT, "yolo: too many priors for one call");
    int32_t* flag = Y.ar.get<int32_t>(90, total);
    int32_t* incl = Y.ar.get<int32_t>(91, total);
    k_yolo_flag<<<cdiv(total, 256), 256, 0, st>>>(d, total, flag);
    inclusive_scan_i32(Y.ar, 92, flag, incl, total, st);
    int32_t* dcnt = Y.ar.get<int32_t>(93, B);
    k_yolo_counts<<<cdiv(B, 64), 64, 0, st>>>(incl, d.dim, B, dcnt);
    std::vector<int32_t> cnt(B);
    VTF_HIP(hipMemcpyAsync(cnt.data(), dcnt, B * 4, hipMemcpyDeviceToHost, st));
    VTF_HIP(hipStreamSynchronize(st));
    int64_t n = 0;
    std::vector<int64_t> calls(B);
    for (int b = 0; b < B; b++) n += calls[b] = cnt[b];
    out.counts.assign(B, 0);
    out.rows.clear();
    out.d_rows = nullptr;
    out.n = 0;
    if (n == 0) return;
    float4* boxes = Y.ar.get<float4>(94, n);
    float* score = Y.ar.get<float>(95, n);
    int32_t* call = Y.ar.get<int32_t>(96, n);
    int32_t* cls = Y.ar.get<int32_t>(97, n);
    k_yolo_emit<<<cdiv(total, 256), 256, 0, st>>>(d, total, flag, incl, boxes, score, call, cls);
    int32_t* keep = Y.ar.get<int32_t>(98, n);
    std::vector<int64_t> nk;
    nms_multi(Y.ar, (const float*)boxes, score, cls, call, calls, 1, 0.45, keep, nk, st);
    const int top = 100;
    std::vector<int64_t> offs(3 * (size_t)B);
    int64_t kb = 0, ob = 0;
    for (int b = 0; b < B; b++) {
        offs[3 * b] = kb;
        offs[3 * b + 1] = std::min<int64_t>(nk[b], top);
        offs[3 * b + 2] = ob;
        out.counts[b] = (int32_t)offs[3 * b + 1];
        kb += nk[b];
        ob += offs[3 * b + 1];
    }
    int64_t* doffs = Y.ar.get<int64_t>(99, 3 * (size_t)B);
    VTF_HIP(hipMemcpyAsync(doffs, offs.data(), offs.size() * 8, hipMemcpyHostToDevice, st));
    float* drows = Y.ar.get<float>(100, std::max<int64_t>(ob, 1) * 5);
    int h, w;
    used_size(H, W, h, w);
    // scale_boxes: torch.tensor(szo) / torch.tensor(szu) in fp32, flipped to (x, y)
    float sx = (float)W / (float)w, sy = (float)H / (float)h;
    k_yolo_final<<<B, 128, 0, st>>>(keep, doffs, boxes, score, sx, sy, top, drows);
    out.d_rows = drows;
    out.n = ob;
    if (!out.host) return;
    out.rows.resize((size_t)ob * 5);
    VTF_HIP(hipMemcpyAsync(out.rows.data(), drows, ob * 20, hipMemcpyDeviceToHost, st));
    VTF_HIP(hipStreamSynchronize(st));
}

static void maps_alloc(Yolo& Y, int B, int Hp, int Wp, float* maps[3]) {
    const int s[3] = {32, 16, 8};
    for (int i = 0; i < 3; i++) maps[i] = Y.ar.get<float>(101 + i, (size_t)B * (Hp / s[i]) * (Wp / s[i]) * 18);
}

static void detect(Yolo& Y, const uint8_t* frames, int on_dev, int B, int H, int W, int64_t fstride, int64_t rstride,
                   YOut& out) {
    VTF_CHECK(B > 0 && H > 0 && W > 0, VTF_E_ARG, "yolo: bad shape");
    hipStream_t st = Y.st;
    const uint8_t* fr = frames;
    if (!on_dev) {
        uint8_t* d = Y.ar.get<uint8_t>(104, (size_t)B * H * W * 3);
        for (int b = 0; b < B; b++)
            VTF_HIP(hipMemcpy2DAsync(d + (size_t)b * H * W * 3, (size_t)W * 3, frames + b * fstride, rstride,
                                     (size_t)W * 3, H, hipMemcpyHostToDevice, st));
        fr = d;
        fstride = (int64_t)H * W * 3;
        rstride = (int64_t)W * 3;
    }
    int h, w;
    used_size(H, W, h, w);
    const int Hp = (h + 31) / 32 * 32, Wp = (w + 31) / 32 * 32;
    float* maps[3];
    if (Y.x3 && stem_on()) {
        maps_alloc(Y, B, Hp, Wp, maps);
        const YStemIn si{fr, fstride, rstride, H, W, h, w};
        net(Y, nullptr, B, Hp, Wp, maps, &si);
    } else {
        void* x0 = Y.ar.get(105, (size_t)B * Hp * Wp * 8 * Y.es());
        launch_letterbox(fr, fstride, rstride, B, H, W, h, w, Hp, Wp, Y.bf16, x0, st, Y.x3);
        maps_alloc(Y, B, Hp, Wp, maps);
        net(Y, x0, B, Hp, Wp, maps);
    }
    postprocess(Y, maps, B, Hp, Wp, H, W, out);
}

static void write_out(const YOut& r, int B, float* out_boxes, float* out_scores, int32_t* out_counts, int64_t cap,
                      int64_t* out_total) {
    int64_t n = (int64_t)r.rows.size() / 5;
    if (out_total) *out_total = n;
    VTF_CHECK(n <= cap, VTF_E_CAPACITY, "output capacity too small");
    for (int b = 0; b < B; b++) out_counts[b] = r.counts[b];
    for (int64_t e = 0; e < n; e++) {
        if (out_boxes) std::memcpy(out_boxes + e * 4, &r.rows[e * 5], 16);
        if (out_scores) out_scores[e] = r.rows[e * 5 + 4];
    }
}

}  // namespace vtf

using namespace vtf;

struct vtf_yolo_s {
    Yolo y;
};

extern "C" {

int vtf_yolo_create(const float* params, int64_t n_params, int device, int precision, vtf_yolo_t* out) {
    return guarded([&] {
        VTF_CHECK(params && out && precision >= 0 && precision <= 2, VTF_E_ARG,
                  "bad argument (precision 0 fp32, 1 bf16, 2 bf16x3)");
        DeviceGuard dg(device);
        auto* h = new vtf_yolo_s();
        h->y.device = device;
        h->y.bf16 = precision == 1;
        h->y.x3 = precision == 2;
        try {
            build(h->y, params, n_params);
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
    });
}

int vtf_yolo_destroy(vtf_yolo_t h) {
    return guarded_on(h ? h->y.device : -1, [&] { delete h; });
}

int vtf_yolo_set_stream(vtf_yolo_t h, void* stream) {
    return guarded_on(h ? h->y.device : -1, [&] {
        VTF_CHECK(h, VTF_E_ARG, "null handle");
        h->y.st = (hipStream_t)stream;
    });
}

int vtf_yolo_detect(vtf_yolo_t h, const uint8_t* frames, int frames_on_device, int B, int H, int W,
                    int64_t frame_stride, int64_t row_stride, float* out_boxes, float* out_scores, int32_t* out_counts,
                    int64_t cap, int64_t* out_total) {
    return guarded_on(h ? h->y.device : -1, [&] {
        VTF_CHECK(h && frames && out_counts, VTF_E_ARG, "null argument");
        YOut r;
        detect(h->y, frames, frames_on_device, B, H, W, frame_stride, row_stride, r);
        write_out(r, B, out_boxes, out_scores, out_counts, cap, out_total);
    });
}

int vtf_yolo_detect_crops(vtf_yolo_t h, const uint8_t* frames, int frames_on_device, int B, int H, int W,
                          int64_t frame_stride, int64_t row_stride, const vtf_box_params* params,
                          int32_t frame_offset, int32_t* d_crops, int32_t* out_frame_counts, int64_t cap,
                          int64_t* out_n) {
    return guarded_on(h ? h->y.device : -1, [&] {
        VTF_CHECK(h && frames && params && out_n, VTF_E_ARG, "null argument");
        YOut r;
        r.host = false;
        detect(h->y, frames, frames_on_device, B, H, W, frame_stride, row_stride, r);
        VTF_CHECK(r.n == 0 || d_crops, VTF_E_ARG, "null argument");
        rows_to_crops(h->y.ar, 110, r.d_rows, r.counts, H, W, *params, frame_offset, d_crops, nullptr,
                      out_frame_counts, cap, out_n, h->y.st);
    });
}

int vtf_yolo_input_size(int H, int W, int* out4) {
    return guarded([&] {
        VTF_CHECK(out4 && H > 0 && W > 0, VTF_E_ARG, "bad argument");
        int h, w;
        used_size(H, W, h, w);
        out4[0] = h;
        out4[1] = w;
        out4[2] = (h + 31) / 32 * 32;
        out4[3] = (w + 31) / 32 * 32;
    });
}

int vtf_yolo_letterbox(vtf_yolo_t h, const uint8_t* d_frames, int B, int H, int W, int64_t frame_stride,
                       int64_t row_stride, float* d_out) {
    return guarded_on(h ? h->y.device : -1, [&] {
        VTF_CHECK(h && d_frames && d_out && B > 0, VTF_E_ARG, "bad argument");
        int hh, ww;
        used_size(H, W, hh, ww);
        launch_letterbox(d_frames, frame_stride, row_stride, B, H, W, hh, ww, (hh + 31) / 32 * 32,
                         (ww + 31) / 32 * 32, false, d_out, h->y.st);
        VTF_HIP(hipStreamSynchronize(h->y.st));
    });
}

int vtf_yolo_net(vtf_yolo_t h, const float* d_x, int B, int Hp, int Wp, float* d_map0, float* d_map1, float* d_map2) {
    return guarded_on(h ? h->y.device : -1, [&] {
        VTF_CHECK(h && d_x && d_map0 && d_map1 && d_map2 && B > 0, VTF_E_ARG, "bad argument");
        Yolo& Y = h->y;
        void* x0 = Y.ar.get(105, (size_t)B * Hp * Wp * 8 * Y.es());
        if (Y.x3)
            k_nchw_to_s3<<<cdiv((int64_t)B * Hp * Wp, 256), 256, 0, Y.st>>>(d_x, B, 3, Hp, Wp, (char*)x0);
        else
            launch_nchw_to_nhwc(d_x, B, 3, Hp, Wp, 8, x0, Y.bf16, Y.st);
        float* maps[3] = {d_map0, d_map1, d_map2};
        net(Y, x0, B, Hp, Wp, maps);
        VTF_HIP(hipStreamSynchronize(Y.st));
    });
}

int vtf_yolo_postprocess(vtf_yolo_t h, const float* d_map0, const float* d_map1, const float* d_map2, int B, int H,
                         int W, float* out_boxes, float* out_scores, int32_t* out_counts, int64_t cap,
                         int64_t* out_total) {
    return guarded_on(h ? h->y.device : -1, [&] {
        VTF_CHECK(h && d_map0 && d_map1 && d_map2 && out_counts && B > 0, VTF_E_ARG, "bad argument");
        int hh, ww;
        used_size(H, W, hh, ww);
        float* maps[3] = {(float*)d_map0, (float*)d_map1, (float*)d_map2};
        YOut r;
        postprocess(h->y, maps, B, (hh + 31) / 32 * 32, (ww + 31) / 32 * 32, H, W, r);
        write_out(r, B, out_boxes, out_scores, out_counts, cap, out_total);
    });
}

int vtf_yolo_profile(vtf_yolo_t h, int enable, double* out_ms, int64_t* out_launches, double* out_flops,
                     int64_t* out_frames) {
    return guarded_on(h ? h->y.device : -1, [&] {
        VTF_CHECK(h, VTF_E_ARG, "null handle");
        Yolo& Y = h->y;
        if (out_ms) *out_ms = Y.prof_ms;
        if (out_launches) *out_launches = Y.prof_launches;
        if (out_flops) *out_flops = Y.prof_flops;
        if (out_frames) *out_frames = Y.prof_frames;
        Y.prof_ms = Y.prof_flops = 0;
        Y.prof_launches = Y.prof_frames = 0;
        if (enable) {
            if (!Y.ev0) VTF_HIP(hipEventCreate(&Y.ev0));
            if (!Y.ev1) VTF_HIP(hipEventCreate(&Y.ev1));
        }
        Y.prof = enable != 0;
    });
}

}  // extern "C"

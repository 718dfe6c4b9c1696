// Faster R-CNN anime-face detector (src/videotofaces/detectors/rcnn.py:16-177) on gfx950.
//
//   prep   k_rcnn_prep: cv2 INTER_LINEAR keep-ratio resize to (800, 1333) + BGR->RGB +
//          (x - mean) / std + zero pad to a multiple of 32 (prep.py:12-92), one pass from the
//          uint8 frames in HBM to the NHWC (C padded to 8) network input.
//   body   ResNet50 (backbones/resnet.py:11-54): 53 ConvUnits, each one launch of the
//          implicit-GEMM MFMA kernel (conv.hip) with BN folded and ReLU + the bottleneck
//          residual fused in the epilogue; the 3x3/2 pad-1 stem max-pool is k_maxpool_pad.
//   fpn    1x1 laterals with the top-down nearest-x2 add fused in the epilogue (res_up2:
//          P[i] += interpolate(P[i+1]), rcnn.py:23-31), 3x3 smooths, P6 = P5[::2, ::2].
//   rpn    per level: 3x3 conv + ReLU, ONE 1x1 conv emitting the 3 logits and 12 deltas
//          (fp32); per-(image, level) top-1000 by one segmented radix sort (key = image,
//          level, descending logit); k_rpn_decode (decode_boxes, sigmoid, clamp_to_canvas,
//          remove_small); batched_nms(0.7) over (image, level) groups (nms.hip); first 1000
//          per image (rcnn.py:49-82).
//   roi    k_roi_align: FPN level (roi.py:7-16) + torchvision RoIAlign (7x7, adaptive grid,
//          aligned) per proposal from the NHWC maps -> [R,7,7,256]; FC 12544->1024->1024
//          (ReLU) and one 6-row head (4 deltas, 2 logits) on the MFMA kernel; k_roi_post
//          (softmax, > 0.05, decode (0.1, 0.2), clamp, remove_small) -> per-image nms(0.5)
//          [:100] -> scale_boxes (rcnn.py:103-124, 148-149).
// Build with -ffp-contract=off: box math and RoIAlign round like the reference CPU path.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <vector>

#include "blob.hpp"
#include "boxes.hpp"
#include "common.hpp"
#include "conv.hpp"
#include "nms.hpp"

namespace vtf {

struct RUnit {
    int cin, cout, k, s, p, cin_pad;
    void* w;       // [cout][k][k][cin_pad], element = precision
    float* alpha;  // folded BN (ConvUnit)
    float* beta;
    float* bias;
};

struct RBlock {
    int u1, u2, u3, ds;  // unit indices (ds = -1: identity shortcut)
    int stride, width;
};

struct Rcnn {
    int device = 0;
    bool bf16 = false;
    hipStream_t st = 0;
    std::vector<RUnit> U;
    std::vector<RBlock> blocks[4];
    int i_lat = 0, i_smooth = 0, i_rpn = 0, i_fc = 0;
    std::vector<void*> allocs;
    Arena ar;
    bool prof = false;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double prof_ms = 0, prof_flops = 0, flops = 0;
    int64_t prof_launches = 0, prof_frames = 0, launches = 0;
    std::vector<float> last_props;  // [n,5] (image, x1, y1, x2, y2) of the last detect
    ~Rcnn() {
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
    void* upload_w(const std::vector<float>& w) {
        if (!bf16) return upload(w);
        std::vector<uint16_t> b(w.size());
        for (size_t i = 0; i < w.size(); i++) b[i] = f2bf(w[i]);
        return upload(b);
    }
};

constexpr int R_LEVELS = 5, R_TOP = 1000, R_FINAL = 100;
static const int kStride[R_LEVELS] = {4, 8, 16, 32, 64};

// ------------------------------------------------------------------ weights
static void build(Rcnn& R, const float* params, int64_t n_params) {
    int64_t src = 0;
    auto take = [&](int64_t n) {
        VTF_CHECK(src + n <= n_params, VTF_E_ARG, "rcnn: parameter buffer too small");
        const float* p = params + src;
        src += n;
        return p;
    };
    // conv weight [cout][cin][k][k] -> [cout][k][k][cin_pad]
    auto relayout = [&](const float* w, int cin, int cout, int k, int cin_pad) {
        int K = k * k * cin_pad;
        std::vector<float> wt((size_t)cout * K, 0.f);
        for (int co = 0; co < cout; co++)
            for (int ci = 0; ci < cin; ci++)
                for (int y = 0; y < k; y++)
                    for (int x = 0; x < k; x++)
                        wt[(size_t)co * K + (y * k + x) * cin_pad + ci] = w[(((size_t)co * cin + ci) * k + y) * k + x];
        return wt;
    };
    auto unit = [&](int cin, int cout, int k, int s, int p, bool bn) {
        RUnit u{};
        u.cin = cin;
        u.cout = cout;
        u.k = k;
        u.s = s;
        u.p = p;
        u.cin_pad = (cin + 7) / 8 * 8;
        u.w = R.upload_w(relayout(take((int64_t)cout * cin * k * k), cin, cout, k, u.cin_pad));
        if (bn) {
            // BatchNorm2d(eps 1e-5) folded like torch's CPU inference kernel
            const float* bw = take(cout);
            const float* bb = take(cout);
            const float* bm = take(cout);
            const float* bv = take(cout);
            std::vector<float> a(cout), be(cout);
            for (int c = 0; c < cout; c++) {
                float invstd = 1.f / std::sqrt(bv[c] + 1e-5f);
                a[c] = invstd * bw[c];
                be[c] = bb[c] - bm[c] * a[c];
            }
            u.alpha = R.upload(a);
            u.beta = R.upload(be);
        } else {
            const float* b = take(cout);
            u.bias = R.upload(std::vector<float>(b, b + cout));
        }
        R.U.push_back(u);
        return (int)R.U.size() - 1;
    };
    unit(3, 64, 7, 2, 3, true);  // body.layers.0.0 (resnet.py:42)
    int cin = 64;
    const int widths[4] = {64, 128, 256, 512}, counts[4] = {3, 4, 6, 3};
    for (int li = 0; li < 4; li++) {
        const int w = widths[li];
        for (int b = 0; b < counts[li]; b++) {
            RBlock blk{};
            blk.stride = (b == 0 && li > 0) ? 2 : 1;
            blk.width = w;
            blk.u1 = unit(cin, w, 1, 1, 0, true);
            blk.u2 = unit(w, w, 3, blk.stride, 1, true);  // stride on the 3x3 (resnet.py:18)
            blk.u3 = unit(w, 4 * w, 1, 1, 0, true);
            blk.ds = (blk.stride > 1 || cin != 4 * w) ? unit(cin, 4 * w, 1, blk.stride, 0, true) : -1;
            R.blocks[li].push_back(blk);
            cin = 4 * w;
        }
    }
    const int cins[4] = {256, 512, 1024, 2048};
    R.i_lat = (int)R.U.size();
    for (int i = 0; i < 4; i++) unit(cins[i], 256, 1, 1, 0, false);  // fpn.conv_laterals
    R.i_smooth = (int)R.U.size();
    for (int i = 0; i < 4; i++) unit(256, 256, 3, 1, 1, false);  // fpn.conv_smooths
    R.i_rpn = unit(256, 256, 3, 1, 1, false);                    // rpn.conv
    {
        // rpn.log (3) + rpn.reg (12) as one 15-row 1x1 conv: rows 0-2 logits, 3-14 deltas
        const float* lw = take(3 * 256);
        const float* lb = take(3);
        const float* rw = take(12 * 256);
        const float* rb = take(12);
        std::vector<float> w(15 * 256), b(15);
        std::memcpy(w.data(), lw, 3 * 256 * 4);
        std::memcpy(w.data() + 3 * 256, rw, 12 * 256 * 4);
        std::memcpy(b.data(), lb, 12);
        std::memcpy(b.data() + 3, rb, 48);
        RUnit u{256, 15, 1, 1, 0, 256, R.upload_w(w), nullptr, nullptr, R.upload(b)};
        R.U.push_back(u);
    }
    R.i_fc = (int)R.U.size();
    {
        // roi.fc.0 over the flattened [256,7,7] RoI maps (c, ph, pw); the RoI maps here are
        // NHWC [7,7,256], so the weight columns are permuted to (ph, pw, c)
        const float* w = take((int64_t)1024 * 12544);
        const float* b = take(1024);
        std::vector<float> wt((size_t)1024 * 12544);
        for (int o = 0; o < 1024; o++)
            for (int c = 0; c < 256; c++)
                for (int q = 0; q < 49; q++) wt[(size_t)o * 12544 + q * 256 + c] = w[(size_t)o * 12544 + c * 49 + q];
        RUnit u{12544, 1024, 1, 1, 0, 12544, R.upload_w(wt), nullptr, nullptr, R.upload(std::vector<float>(b, b + 1024))};
        R.U.push_back(u);
    }
    {
        const float* w = take((int64_t)1024 * 1024);
        const float* b = take(1024);
        RUnit u{1024, 1024, 1, 1, 0, 1024, R.upload_w(std::vector<float>(w, w + (size_t)1024 * 1024)), nullptr,
                nullptr, R.upload(std::vector<float>(b, b + 1024))};
        R.U.push_back(u);
    }
    {
        // roi.cls (2) + roi.reg (4) as one 6-row head: rows 0-3 deltas, 4-5 logits
        const float* cw = take(2 * 1024);
        const float* cb = take(2);
        const float* rw = take(4 * 1024);
        const float* rb = take(4);
        std::vector<float> w(6 * 1024), b(6);
        std::memcpy(w.data(), rw, 4 * 1024 * 4);
        std::memcpy(w.data() + 4 * 1024, cw, 2 * 1024 * 4);
        std::memcpy(b.data(), rb, 16);
        std::memcpy(b.data() + 4, cb, 8);
        RUnit u{1024, 6, 1, 1, 0, 1024, R.upload_w(w), nullptr, nullptr, R.upload(b)};
        R.U.push_back(u);
    }
    VTF_CHECK(src == n_params, VTF_E_ARG, "rcnn: expected 41,401,301 parameters");
}

// ------------------------------------------------------------------ preprocess
// resize_cv2 keep-ratio size for resize=(800, 1333) in Python doubles (prep.py:71-74)
static void used_size(int H, int W, int& h, int& w) {
    double scl = std::min(800.0 / std::min(H, W), 1333.0 / std::max(H, W));
    h = (int)(H * scl + 0.5);
    w = (int)(W * scl + 0.5);
}

template <typename T>
__global__ void k_rcnn_prep(const uint8_t* __restrict__ frames, int64_t fstride, int64_t rstride, int H, int W, int h,
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
        // to_tensors(means='imagenet', stdvs='imagenet', to_rgb=True): t -= mean; t /= std
        const float mean[3] = {123.675f, 116.28f, 103.53f}, stdv[3] = {58.395f, 57.12f, 57.375f};
        for (int oc = 0; oc < 3; oc++) v[oc] = __fdiv_rn((float)u[2 - oc] - mean[oc], stdv[oc]);
    }
    T* o = out + i * 8;
#pragma unroll
    for (int c = 0; c < 8; c++) o[c] = (T)v[c];
}

static void launch_prep(const uint8_t* frames, int64_t fstride, int64_t rstride, int B, int H, int W, int h, int w,
                        int Hp, int Wp, bool bf16, void* out, hipStream_t st) {
    int64_t total = (int64_t)B * Hp * Wp;
    if (bf16)
        k_rcnn_prep<__bf16><<<cdiv(total, 256), 256, 0, st>>>(frames, fstride, rstride, H, W, h, w, Hp, Wp, total,
                                                               (__bf16*)out);
    else
        k_rcnn_prep<float><<<cdiv(total, 256), 256, 0, st>>>(frames, fstride, rstride, H, W, h, w, Hp, Wp, total,
                                                              (float*)out);
}

// ------------------------------------------------------------------ small layout kernels
__device__ inline float ldf(const float* p) { return *p; }
__device__ inline float ldf(const __bf16* p) { return (float)*p; }

// MaxPool2d(3, 2, padding=1) NHWC (resnet.py:43); padding never wins (-inf)
template <typename T>
__global__ void k_maxpool_pad(const T* __restrict__ in, int N, int H, int W, int C, int OH, int OW, T* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t tot = (int64_t)N * OH * OW * C;
    if (i >= tot) return;
    int c = (int)(i % C);
    int64_t t = i / C;
    int ow = (int)(t % OW);
    t /= OW;
    int oh = (int)(t % OH);
    int n = (int)(t / OH);
    float m = -INFINITY;
    for (int dy = 0; dy < 3; dy++) {
        int y = 2 * oh - 1 + dy;
        if (y < 0 || y >= H) continue;
        for (int dx = 0; dx < 3; dx++) {
            int x = 2 * ow - 1 + dx;
            if (x < 0 || x >= W) continue;
            m = fmaxf(m, ldf(in + (((int64_t)n * H + y) * W + x) * C + c));
        }
    }
    out[i] = (T)m;
}

// max_pool2d(P5, 1, stride=2) == P5[:, ::2, ::2] (rcnn.py:30)
template <typename T>
__global__ void k_subsample2(const T* __restrict__ in, int N, int H, int W, int C, int OH, int OW, T* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t tot = (int64_t)N * OH * OW * C;
    if (i >= tot) return;
    int c = (int)(i % C);
    int64_t t = i / C;
    int ow = (int)(t % OW);
    t /= OW;
    int oh = (int)(t % OH);
    int n = (int)(t / OH);
    out[i] = in[(((int64_t)n * H + 2 * oh) * W + 2 * ow) * C + c];
}

// ------------------------------------------------------------------ net
static void cunit(Rcnn& R, int ui, const void* in, int N, int H, int W, void* out, int out_cs, bool relu,
                  const void* res = nullptr, int res_cs = 0, bool res_up2 = false, bool out_f32 = false) {
    const RUnit& u = R.U[ui];
    ConvParams p{};
    p.in = in;
    p.w = u.w;
    p.out = out;
    p.N = N;
    p.H = H;
    p.W = W;
    p.Cin = u.cin_pad;
    p.KH = p.KW = u.k;
    p.sh = p.sw = u.s;
    p.ph = p.pw = u.p;
    p.OH = (H + 2 * u.p - u.k) / u.s + 1;
    p.OW = (W + 2 * u.p - u.k) / u.s + 1;
    p.Cout = u.cout;
    p.K = u.k * u.k * u.cin_pad;
    p.M = (int64_t)N * p.OH * p.OW;
    p.out_cstride = out_cs;
    p.scale = 1.f;
    p.bias = u.bias;
    p.alpha = u.alpha;
    p.beta = u.beta;
    p.relu = relu ? 1 : 0;
    if (res) {
        p.res = res;
        p.res_cstride = res_cs;
        p.res_up2 = res_up2 ? 1 : 0;
    }
    p.out_f32 = out_f32 ? 1 : 0;
    launch_conv(p, R.bf16, R.st);
    R.flops += 2.0 * (double)p.M * u.cout * u.k * u.k * u.cin;
    R.launches++;
}

struct RMap {
    void* p;
    int h, w;
};

// x0 NHWC [B,Hp,Wp,8] -> P2..P6 (NHWC, 256 ch) and the RPN head maps (NHWC fp32 [B,h,w,15])
static void net(Rcnn& R, const void* x0, int B, int Hp, int Wp, RMap P[R_LEVELS], float* heads[R_LEVELS]) {
    VTF_CHECK(Hp % 32 == 0 && Wp % 32 == 0 && Hp > 0 && Wp > 0, VTF_E_ARG, "rcnn: input must be padded to x32");
    const size_t es = R.bf16 ? 2 : 4;
    hipStream_t st = R.st;
    R.flops = 0;
    R.launches = 0;
    if (R.prof) VTF_HIP(hipEventRecord(R.ev0, st));
    const int H1 = Hp / 2, W1 = Wp / 2, H2 = Hp / 4, W2 = Wp / 4;
    const size_t big = (size_t)B * H2 * W2 * 256 * es;  // largest block tensor (layer 1 output)
    char* S = (char*)R.ar.get(200, (size_t)B * H1 * W1 * 64 * es);
    char* A = (char*)R.ar.get(201, big);
    char* Bf = (char*)R.ar.get(202, big);
    char* T1 = (char*)R.ar.get(203, big / 2);  // u1 out: <= H2*W2*128
    char* T2 = (char*)R.ar.get(204, big / 4);  // u2 out: <= H2*W2*64
    char* D = (char*)R.ar.get(205, big);       // downsample out
    cunit(R, 0, x0, B, Hp, Wp, S, 64, true);
    {
        int64_t tot = (int64_t)B * H2 * W2 * 64;
        if (R.bf16)
            k_maxpool_pad<__bf16><<<cdiv(tot, 256), 256, 0, st>>>((const __bf16*)S, B, H1, W1, 64, H2, W2, (__bf16*)A);
        else
            k_maxpool_pad<float><<<cdiv(tot, 256), 256, 0, st>>>((const float*)S, B, H1, W1, 64, H2, W2, (float*)A);
    }
    RMap C[4];
    const char* cur = A;
    int h = H2, w = W2, c = 64;
    for (int li = 0; li < 4; li++) {
        const int nb = (int)R.blocks[li].size();
        for (int bi = 0; bi < nb; bi++) {
            const RBlock& k = R.blocks[li][bi];
            const int ho = (h - 1) / k.stride + 1, wo = (w - 1) / k.stride + 1;
            const int co = 4 * k.width;
            const void* res = cur;
            if (k.ds >= 0) {
                cunit(R, k.ds, cur, B, h, w, D, co, false);
                res = D;
            }
            cunit(R, k.u1, cur, B, h, w, T1, k.width, true);
            cunit(R, k.u2, T1, B, h, w, T2, k.width, true);
            char* out;
            if (bi == nb - 1) {
                out = (char*)R.ar.get(210 + li, (size_t)B * ho * wo * co * es);
            } else {
                out = (cur == A) ? Bf : A;
            }
            cunit(R, k.u3, T2, B, ho, wo, out, co, true, res, co);  // relu(bn(conv) + shortcut)
            cur = out;
            h = ho;
            w = wo;
            c = co;
        }
        C[li] = {(void*)cur, h, w};
    }
    (void)c;
    // FPN (rcnn.py:23-31): laterals top-down with the x2 nearest add fused, then smooths
    char* Lat[4];
    for (int i = 3; i >= 0; i--) {
        Lat[i] = (char*)R.ar.get(220 + i, (size_t)B * C[i].h * C[i].w * 256 * es);
        if (i == 3)
            cunit(R, R.i_lat + i, C[i].p, B, C[i].h, C[i].w, Lat[i], 256, false);
        else
            cunit(R, R.i_lat + i, C[i].p, B, C[i].h, C[i].w, Lat[i], 256, false, Lat[i + 1], 256, true);
    }
    for (int i = 0; i < 4; i++) {
        P[i] = {R.ar.get(230 + i, (size_t)B * C[i].h * C[i].w * 256 * es), C[i].h, C[i].w};
        cunit(R, R.i_smooth + i, Lat[i], B, C[i].h, C[i].w, P[i].p, 256, false);
    }
    {
        const int oh = (P[3].h - 1) / 2 + 1, ow = (P[3].w - 1) / 2 + 1;
        P[4] = {R.ar.get(234, (size_t)B * oh * ow * 256 * es), oh, ow};
        int64_t tot = (int64_t)B * oh * ow * 256;
        if (R.bf16)
            k_subsample2<__bf16><<<cdiv(tot, 256), 256, 0, st>>>((const __bf16*)P[3].p, B, P[3].h, P[3].w, 256, oh, ow,
                                                                  (__bf16*)P[4].p);
        else
            k_subsample2<float><<<cdiv(tot, 256), 256, 0, st>>>((const float*)P[3].p, B, P[3].h, P[3].w, 256, oh, ow,
                                                                 (float*)P[4].p);
    }
    // RPN head per level (rcnn.py:42-47)
    for (int l = 0; l < R_LEVELS; l++) {
        cunit(R, R.i_rpn, P[l].p, B, P[l].h, P[l].w, A, 256, true);
        cunit(R, R.i_rpn + 1, A, B, P[l].h, P[l].w, heads[l], 15, false, nullptr, 0, false, true);
    }
    if (R.prof) {
        VTF_HIP(hipEventRecord(R.ev1, st));
        VTF_HIP(hipEventSynchronize(R.ev1));
        float ms = 0;
        VTF_HIP(hipEventElapsedTime(&ms, R.ev0, R.ev1));
        R.prof_ms += ms;
        R.prof_flops += R.flops;
        R.prof_launches += R.launches;
        R.prof_frames += B;
    }
}

// ------------------------------------------------------------------ RPN proposals
struct RLevel {
    const float* head;  // NHWC fp32 [B,h,w,15]
    int h, w, stride;
    int64_t L, off;     // priors of the level per image, prefix within the image
    int64_t top, toff;  // min(1000, L), prefix of the tops
    float aw[3], ah[3];
};
struct RDec {
    RLevel lv[R_LEVELS];
    int64_t Ltot, dim;
    float wu, hu;  // used (unpadded) image size: clamp_to_canvas bounds
    // CPU threads of the reference run whose sigmoid rounding is reproduced (torch_sigmoid): it
    // only matters above 32768 objectness values (det-batch >= 7); VTF_TORCH_THREADS, default 8
    // (the survey container that made the goldens)
    int torch_threads;
};

__device__ inline int level_of(const RDec& d, int64_t r, bool tops) {
    int l = 0;
    for (int k = 1; k < R_LEVELS; k++)
        if (r >= (tops ? d.lv[k].toff : d.lv[k].off)) l = k;
    return l;
}

// key = [image*5 + level : 32][descending logit : 32], value = prior index within the level
__global__ void k_rpn_keys(RDec d, int64_t total, uint64_t* __restrict__ keys, int32_t* __restrict__ vals) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= total) return;
    int64_t b = i / d.Ltot, r = i % d.Ltot;
    int l = level_of(d, r, false);
    const RLevel& L = d.lv[l];
    int64_t p = r - L.off;
    int64_t cell = p / 3;
    int a = (int)(p % 3);
    float logit = L.head[(b * L.h * L.w + cell) * 15 + a];
    keys[i] = ((uint64_t)(b * R_LEVELS + l) << 32) | desc_key(logit);
    vals[i] = (int32_t)p;
}

// torch's CPU sigmoid, bit for bit (rcnn.py:68 `torch.cat(logits).sigmoid()`): ATen's
// sigmoid_kernel runs 1 / (1 + exp(-x)) with Vectorized<float>::exp = Sleef_expf16_u10 on the
// 32-element vector steps of every parallel_for chunk and the scalar lambda (std::exp = glibc
// expf) on each chunk's last (len % 32) elements; chunks = divup(numel, min(threads,
// divup(numel, 32768))).  Measured in the survey container (AVX512 capability; the Sleef
// routine disassembled from libtorch_cpu.so, constants read from the binary) and matched bit for
// bit over 4e5 random logits (scripts/torch_sigmoid_order.py).
__device__ inline float sleef_expf_u10(float d) {
    const float q = rintf(d * 1.44269502162933349609375f);  // vcvtps2dq: round to nearest even
    float s = fmaf(q, -0.693145751953125f, d);
    s = fmaf(q, -1.428606765330187045e-06f, s);
    float u = 0.000198527617612853646278381f;
    u = fmaf(s, u, 0.00139304355252534151077271f);
    u = fmaf(s, u, 0.00833336077630519866943359f);
    u = fmaf(s, u, 0.0416664853692054748535156f);
    u = fmaf(s, u, 0.166666671633720397949219f);
    u = fmaf(s, u, 0.5f);
    u = fmaf(s * s, u, s);
    u = u + 1.0f;
    const int qi = (int)q, h = qi >> 1;
    u *= __int_as_float((h + 127) << 23);
    u *= __int_as_float((qi - h + 127) << 23);
    if (d < -104.f) u = 0.f;
    if (100.f < d) u = INFINITY;
    return u;
}

// glibc 2.35 expf (sysdeps/ieee754/flt-32/e_expf.c, EXP2F_TABLE_BITS 5): double-precision
// k/N + r reduction, table 2^(i/32), cubic polynomial
__constant__ uint64_t GLIBC_EXP2F_TAB[32] = {
    0x3ff0000000000000ull, 0x3fefd9b0d3158574ull, 0x3fefb5586cf9890full, 0x3fef9301d0125b51ull,
    0x3fef72b83c7d517bull, 0x3fef54873168b9aaull, 0x3fef387a6e756238ull, 0x3fef1e9df51fdee1ull,
    0x3fef06fe0a31b715ull, 0x3feef1a7373aa9cbull, 0x3feedea64c123422ull, 0x3feece086061892dull,
    0x3feebfdad5362a27ull, 0x3feeb42b569d4f82ull, 0x3feeab07dd485429ull, 0x3feea47eb03a5585ull,
    0x3feea09e667f3bcdull, 0x3fee9f75e8ec5f74ull, 0x3feea11473eb0187ull, 0x3feea589994cce13ull,
    0x3feeace5422aa0dbull, 0x3feeb737b0cdc5e5ull, 0x3feec49182a3f090ull, 0x3feed503b23e255dull,
    0x3feee89f995ad3adull, 0x3feeff76f2fb5e47ull, 0x3fef199bdd85529cull, 0x3fef3720dcef9069ull,
    0x3fef5818dcfba487ull, 0x3fef7c97337b9b5full, 0x3fefa4afa2a490daull, 0x3fefd0765b6e4540ull};

__device__ inline float glibc_expf(float x) {
    if (x != x) return x + x;
    if (x > 88.72283172607421875f) return INFINITY;    // 0x1.62e42ep6f
    if (x < -103.972076416015625f) return 0.f;         // -0x1.9fe368p6f
    const double xd = (double)x;
    const double z = 46.16624130844682704 * xd;        // 0x1.71547652b82fep+5 = 32 / ln 2
    const double shift = 6755399441055744.0;           // 0x1.8p+52
    double kd = z + shift;
    const uint64_t ki = (uint64_t)__double_as_longlong(kd);
    kd -= shift;
    const double r = z - kd;
    uint64_t t = GLIBC_EXP2F_TAB[ki % 32];
    t += ki << (52 - 5);
    const double sc = __longlong_as_double((long long)t);
    const double zz = fma(1.6938359250920212e-06, r, 0.00023459809789509004);   // C0 r + C1
    const double r2 = r * r;
    double y = fma(0.021660849396613134, r, 1.0);                             // C2 r + 1
    y = fma(zz, r2, y);
    return (float)(y * sc);
}

// element j of a numel-element contiguous float tensor through torch.sigmoid on `threads` CPU
// threads (the reference's own run: the chunk tails take the scalar glibc path)
__device__ inline float torch_sigmoid(float x, int64_t j, int64_t numel, int threads) {
    const int64_t nt = min<int64_t>(threads, (numel + 32767) / 32768);
    const int64_t cs = (numel + nt - 1) / nt;
    const int64_t c0 = (j / cs) * cs, c1 = min(numel, c0 + cs);
    const bool scalar = j >= c1 - (c1 - c0) % 32;
    const float e = scalar ? glibc_expf(-x) : sleef_expf_u10(0.f - x);
    return __fdiv_rn(1.f, 1.f + e);
}

// filt_dec + sigmoid + clamp_to_canvas + remove_small(0) (rcnn.py:49-77; bbox.py:6-60)
__global__ void k_rpn_decode(RDec d, int64_t total, const int32_t* __restrict__ sorted_vals, float4* __restrict__ boxes,
                             float* __restrict__ obj, int32_t* __restrict__ group, int32_t* __restrict__ flag) {
    int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= total) return;
    int64_t b = j / d.dim, r = j % d.dim;
    int l = level_of(d, r, true);
    const RLevel& L = d.lv[l];
    int64_t q = r - L.toff;
    int64_t p = sorted_vals[b * d.Ltot + L.off + q];
    int64_t cell = p / 3;
    int a = (int)(p % 3);
    int x = (int)(cell % L.w), y = (int)(cell / L.w);
    const float* t = L.head + (b * L.h * L.w + cell) * 15;
    float logit = t[a];
    const float* dl = t + 3 + 4 * a;
    // get_priors(loc='corner'): arange * stride (anchor.py:52-58)
    float cx = (float)x * (float)L.stride, cy = (float)y * (float)L.stride;
    float aw = L.aw[a], ah = L.ah[a];
    float X = aw * dl[0] + cx, Y = ah * dl[1] + cy;
    float Wd = aw * expf(dl[2]), Hd = ah * expf(dl[3]);
    float4 bx = make_float4(X - Wd * 0.5f, Y - Hd * 0.5f, X + Wd * 0.5f, Y + Hd * 0.5f);
    bx.x = fminf(fmaxf(bx.x, 0.f), d.wu);
    bx.y = fminf(fmaxf(bx.y, 0.f), d.hu);
    bx.z = fminf(fmaxf(bx.z, 0.f), d.wu);
    bx.w = fminf(fmaxf(bx.w, 0.f), d.hu);
    boxes[j] = bx;
    obj[j] = torch_sigmoid(logit, j, total, d.torch_threads);
    group[j] = (int32_t)(b * 10 + l);
    flag[j] = ((bx.z - bx.x) > 0.f && (bx.w - bx.y) > 0.f) ? 1 : 0;
}

template <class T>
__global__ void k_compact4(const int32_t* __restrict__ flag, const int32_t* __restrict__ incl, int64_t n,
                           const float4* __restrict__ b, const float* __restrict__ s, const T* __restrict__ g,
                           float4* __restrict__ bo, float* __restrict__ so, T* __restrict__ go) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n || !flag[k]) return;
    int64_t o = incl[k] - 1;
    bo[o] = b[k];
    so[o] = s[k];
    go[o] = g[k];
}

static RDec make_rdec(float* const heads[R_LEVELS], const RMap P[R_LEVELS], int h_used, int w_used) {
    RDec d{};
    // make_anchors([32..512], [1], [2, 1, 0.5]): (d*sqrt(r), d/sqrt(r)) in Python doubles
    const double ratios[3] = {2.0, 1.0, 0.5};
    int64_t off = 0, toff = 0;
    for (int l = 0; l < R_LEVELS; l++) {
        RLevel& L = d.lv[l];
        L.head = heads[l];
        L.h = P[l].h;
        L.w = P[l].w;
        L.stride = kStride[l];
        L.L = (int64_t)L.h * L.w * 3;
        L.off = off;
        L.top = std::min<int64_t>(R_TOP, L.L);
        L.toff = toff;
        const double dim = 32.0 * (1 << l);
        for (int a = 0; a < 3; a++) {
            double m = std::sqrt(ratios[a]);
            L.aw[a] = (float)(dim * m);
            L.ah[a] = (float)(dim / m);
        }
        off += L.L;
        toff += L.top;
    }
    d.Ltot = off;
    d.dim = toff;
    d.wu = (float)w_used;
    d.hu = (float)h_used;
    const char* te = std::getenv("VTF_TORCH_THREADS");
    d.torch_threads = te && std::atoi(te) > 0 ? std::atoi(te) : 8;
    return d;
}

// -> proposals (device float4 [n]) + image index (device int32 [n]), reference order
static int64_t rpn_proposals(Rcnn& R, float* const heads[R_LEVELS], const RMap P[R_LEVELS], int B, int hu, int wu,
                             float4** d_props, int32_t** d_pimg) {
    hipStream_t st = R.st;
    RDec d = make_rdec(heads, P, hu, wu);
    const int64_t N = (int64_t)B * d.Ltot;
    VTF_CHECK(N < ((int64_t)1 << 31), VTF_E_LIMIT, "rcnn: too many priors for one call");
    uint64_t* k0 = R.ar.get<uint64_t>(240, N);
    uint64_t* k1 = R.ar.get<uint64_t>(241, N);
    int32_t* v0 = R.ar.get<int32_t>(242, N);
    int32_t* v1 = R.ar.get<int32_t>(243, N);
    k_rpn_keys<<<cdiv(N, 256), 256, 0, st>>>(d, N, k0, v0);
    int seg_bits = 1;
    while ((1ll << seg_bits) < (int64_t)B * R_LEVELS) seg_bits++;
    sort_u64_pairs(R.ar, 244, k0, k1, v0, v1, N, 32 + seg_bits, st);
    const int64_t M = (int64_t)B * d.dim;
    float4* bx = R.ar.get<float4>(245, M);
    float* ob = R.ar.get<float>(246, M);
    int32_t* gr = R.ar.get<int32_t>(247, M);
    int32_t* fl = R.ar.get<int32_t>(248, M);
    int32_t* inc = R.ar.get<int32_t>(249, M);
    k_rpn_decode<<<cdiv(M, 256), 256, 0, st>>>(d, M, v1, bx, ob, gr, fl);
    inclusive_scan_i32(R.ar, 250, fl, inc, M, st);
    int32_t n = 0;
    VTF_HIP(hipMemcpyAsync(&n, inc + M - 1, 4, hipMemcpyDeviceToHost, st));
    VTF_HIP(hipStreamSynchronize(st));
    float4* cb = R.ar.get<float4>(251, std::max(n, 1));
    float* cs = R.ar.get<float>(252, std::max(n, 1));
    int32_t* cg = R.ar.get<int32_t>(253, std::max(n, 1));
    k_compact4<int32_t><<<cdiv(M, 256), 256, 0, st>>>(fl, inc, M, bx, ob, gr, cb, cs, cg);
    // one torchvision batched_nms(0.7) over all images, groups = image * 10 + level (rcnn.py:78-79)
    int32_t* keep = R.ar.get<int32_t>(254, std::max(n, 1));
    int32_t* call = R.ar.get<int32_t>(255, std::max(n, 1));
    VTF_HIP(hipMemsetAsync(call, 0, (size_t)std::max(n, 1) * 4, st));
    std::vector<int64_t> nk;
    nms_multi(R.ar, (const float*)cb, cs, cg, call, {(int64_t)n}, 10 * B, 0.7, keep, nk, st);
    const int64_t kn = nk.empty() ? 0 : nk[0];
    std::vector<int32_t> hk(kn), hg(std::max(n, 1));
    std::vector<float> hs((size_t)std::max(n, 1));
    if (kn) VTF_HIP(hipMemcpyAsync(hk.data(), keep, kn * 4, hipMemcpyDeviceToHost, st));
    if (n) VTF_HIP(hipMemcpyAsync(hg.data(), cg, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    if (n && 4 * (int64_t)n > 4000) VTF_HIP(hipMemcpyAsync(hs.data(), cs, (size_t)n * 4, hipMemcpyDeviceToHost, st));
    VTF_HIP(hipStreamSynchronize(st));
    if (4 * (int64_t)n > 4000) {
        // batched_nms above 4000 coordinates (torchvision ops/boxes.py) returns
        // keep_indices[scores[keep_indices].sort(descending=True)[1]] with keep_indices in index
        // order and torch's default (unstable) CPU sort: std::sort of (score, position) pairs with
        // ATen's KeyValueCompDesc (SortingKernel.cpp) -- its tie order reproduced exactly (checked
        // against torch.sort on tie-heavy inputs, scripts/torch_sigmoid_order.py)
        torch_unstable_desc_order(hk, [&](int32_t e) { return hs[e]; });
    }
    // keep[imidx[keep] == i][:1000] for each image, concatenated (rcnn.py:80)
    std::vector<int32_t> sel, simg;
    std::vector<int> per(B, 0);
    for (int b = 0; b < B; b++)
        for (int64_t t = 0; t < kn; t++) {
            int32_t e = hk[t];
            if (hg[e] / 10 == b && per[b] < R_TOP) {
                sel.push_back(e);
                simg.push_back(b);
                per[b]++;
            }
        }
    const int64_t np = (int64_t)sel.size();
    int32_t* dsel = R.ar.get<int32_t>(256, std::max<int64_t>(np, 1));
    *d_pimg = R.ar.get<int32_t>(257, std::max<int64_t>(np, 1));
    *d_props = R.ar.get<float4>(258, std::max<int64_t>(np, 1));
    if (np) {
        VTF_HIP(hipMemcpyAsync(dsel, sel.data(), np * 4, hipMemcpyHostToDevice, st));
        VTF_HIP(hipMemcpyAsync(*d_pimg, simg.data(), np * 4, hipMemcpyHostToDevice, st));
        std::vector<float4> hb(np);
        // gather on the host copy of the compacted boxes is avoided: one small device gather
        std::vector<float4> all(n);
        VTF_HIP(hipMemcpyAsync(all.data(), cb, (size_t)n * 16, hipMemcpyDeviceToHost, st));
        VTF_HIP(hipStreamSynchronize(st));
        for (int64_t t = 0; t < np; t++) hb[t] = all[sel[t]];
        VTF_HIP(hipMemcpyAsync(*d_props, hb.data(), np * 16, hipMemcpyHostToDevice, st));
        R.last_props.resize(np * 5);
        for (int64_t t = 0; t < np; t++) {
            R.last_props[t * 5] = (float)simg[t];
            R.last_props[t * 5 + 1] = hb[t].x;
            R.last_props[t * 5 + 2] = hb[t].y;
            R.last_props[t * 5 + 3] = hb[t].z;
            R.last_props[t * 5 + 4] = hb[t].w;
        }
    } else {
        R.last_props.clear();
    }
    return np;
}

// ------------------------------------------------------------------ RoIAlign
struct RMaps {
    const void* p[4];
    int h[4], w[4];
    int C;
};

// assign_fpn_levels (roi.py:7-16) + torchvision roi_align(7x7, 1/stride, sampling_ratio 0,
// aligned=True) (roi_align_kernel.cpp) for one proposal per workgroup, one channel per
// thread; out NHWC [R,7,7,C].  Every sample position/weight is wave-uniform scalar math in
// the CPU kernel's evaluation order; the four taps are coalesced channel-vector loads.
template <typename T>
__global__ __launch_bounds__(256) void k_roi_align(RMaps m, const float4* __restrict__ props,
                                                   const int32_t* __restrict__ pimg, int fixed_level, float fixed_scale,
                                                   T* __restrict__ out) {
    const int r = blockIdx.x;
    const float4 bx = props[r];
    const int b = pimg[r];
    int lvl;
    float sc;
    if (fixed_level >= 0) {
        lvl = fixed_level;
        sc = fixed_scale;
    } else {
        float ws = bx.z - bx.x, hs = bx.w - bx.y;
        float k = 4.f + log2f(__fdiv_rn(sqrtf(ws * hs), 224.f));
        k = fminf(fmaxf(k, 2.f), 5.f);
        lvl = (int)(k - 2.f);
        sc = 1.f / (float)(4 << lvl);  // exact
    }
    const int H = m.h[lvl], W = m.w[lvl], C = m.C;
    const T* fm = (const T*)m.p[lvl] + (int64_t)b * H * W * C;
    const float x0 = bx.x * sc - 0.5f, y0 = bx.y * sc - 0.5f;
    const float x1 = bx.z * sc - 0.5f, y1 = bx.w * sc - 0.5f;
    const float rw = x1 - x0, rh = y1 - y0;
    const float bh = __fdiv_rn(rh, 7.f), bw = __fdiv_rn(rw, 7.f);
    const int gh = (int)ceilf(__fdiv_rn(rh, 7.f)), gw = (int)ceilf(__fdiv_rn(rw, 7.f));
    const float cnt = (float)max(gh * gw, 1);
    for (int c = threadIdx.x; c < C; c += blockDim.x) {
        for (int ph = 0; ph < 7; ph++) {
            for (int pw = 0; pw < 7; pw++) {
                float acc = 0.f;
                for (int iy = 0; iy < gh; iy++) {
                    const float yy = (y0 + (float)ph * bh) + __fdiv_rn(((float)iy + 0.5f) * bh, (float)gh);
                    for (int ix = 0; ix < gw; ix++) {
                        const float xx = (x0 + (float)pw * bw) + __fdiv_rn(((float)ix + 0.5f) * bw, (float)gw);
                        float y = yy, x = xx;
                        float w1 = 0.f, w2 = 0.f, w3 = 0.f, w4 = 0.f;
                        int yl = 0, yh = 0, xl = 0, xh = 0;
                        if (!(y < -1.0f || y > (float)H || x < -1.0f || x > (float)W)) {
                            if (y <= 0.f) y = 0.f;
                            if (x <= 0.f) x = 0.f;
                            yl = (int)y;
                            xl = (int)x;
                            if (yl >= H - 1) {
                                yh = yl = H - 1;
                                y = (float)yl;
                            } else {
                                yh = yl + 1;
                            }
                            if (xl >= W - 1) {
                                xh = xl = W - 1;
                                x = (float)xl;
                            } else {
                                xh = xl + 1;
                            }
                            const float ly = y - (float)yl, lx = x - (float)xl;
                            const float hy = 1.f - ly, hx = 1.f - lx;
                            w1 = hy * hx;
                            w2 = hy * lx;
                            w3 = ly * hx;
                            w4 = ly * lx;
                        }
                        const float v1 = ldf(fm + ((int64_t)yl * W + xl) * C + c);
                        const float v2 = ldf(fm + ((int64_t)yl * W + xh) * C + c);
                        const float v3 = ldf(fm + ((int64_t)yh * W + xl) * C + c);
                        const float v4 = ldf(fm + ((int64_t)yh * W + xh) * C + c);
                        acc = acc + (((w1 * v1 + w2 * v2) + w3 * v3) + w4 * v4);
                    }
                }
                out[(((int64_t)r * 7 + ph) * 7 + pw) * C + c] = (T)__fdiv_rn(acc, cnt);
            }
        }
    }
}

static void launch_roi_align(const RMaps& m, const float4* props, const int32_t* pimg, int64_t R, int fixed_level,
                             float fixed_scale, bool bf16, void* out, hipStream_t st) {
    if (R <= 0) return;
    if (bf16)
        k_roi_align<__bf16><<<(unsigned)R, 256, 0, st>>>(m, props, pimg, fixed_level, fixed_scale, (__bf16*)out);
    else
        k_roi_align<float><<<(unsigned)R, 256, 0, st>>>(m, props, pimg, fixed_level, fixed_scale, (float*)out);
}

// ------------------------------------------------------------------ RoI head post-processing
// softmax[:, :-1] > 0.05, convert_to_cwh, decode (0.1, 0.2), clamp, remove_small (rcnn.py:108-122)
__global__ void k_roi_post(const float* __restrict__ hout, const float4* __restrict__ props, int64_t n, float wu,
                           float hu, float4* __restrict__ boxes, float* __restrict__ score, int32_t* __restrict__ flag) {
    int64_t r = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (r >= n) return;
    const float* t = hout + r * 6;
    const float l0 = t[4], l1 = t[5];
    const float mx = fmaxf(l0, l1);
    const float e0 = expf(l0 - mx), e1 = expf(l1 - mx);
    const float s = e0 * __fdiv_rn(1.0f, e0 + e1);
    const float4 p = props[r];
    const float w = p.z - p.x, h = p.w - p.y;
    const float cx = p.x + w * 0.5f, cy = p.y + h * 0.5f;
    const float X = (w * 0.1f) * t[0] + cx, Y = (h * 0.1f) * t[1] + cy;
    const float Wd = w * expf(0.2f * t[2]), Hd = h * expf(0.2f * t[3]);
    float4 bx = make_float4(X - Wd * 0.5f, Y - Hd * 0.5f, X + Wd * 0.5f, Y + Hd * 0.5f);
    bx.x = fminf(fmaxf(bx.x, 0.f), wu);
    bx.y = fminf(fmaxf(bx.y, 0.f), hu);
    bx.z = fminf(fmaxf(bx.z, 0.f), wu);
    bx.w = fminf(fmaxf(bx.w, 0.f), hu);
    boxes[r] = bx;
    score[r] = s;
    flag[r] = (s > 0.05f && (bx.z - bx.x) > 0.f && (bx.w - bx.y) > 0.f) ? 1 : 0;
}

// keep[:100] per image, then scale_boxes (post.py:8, bbox.py:63-67)
__global__ void k_rcnn_final(const int32_t* __restrict__ keep, const int64_t* __restrict__ offs, const float4* boxes,
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

struct ROut {
    std::vector<float> rows;     // [n,5] x1,y1,x2,y2,score (host copy, when requested)
    std::vector<int32_t> counts;  // per image; -1 past the last image holding a proposal
    const float* d_rows = nullptr;  // the same rows in HBM
    int64_t n = 0;
    bool host = true;
};

static void roi_stage(Rcnn& R, const RMap P[R_LEVELS], const float4* d_props, const int32_t* d_pimg, int64_t np, int B,
                      int H, int W, int hu, int wu, ROut& out) {
    hipStream_t st = R.st;
    out.rows.clear();
    out.d_rows = nullptr;
    out.n = 0;
    out.counts.assign(B, 0);
    // n = max(imidx) + 1 (rcnn.py:111): later images are absent from the reference's lists
    int nimg = 0;
    for (int64_t t = 0; t < np; t++) nimg = std::max(nimg, (int)R.last_props[t * 5] + 1);
    for (int b = nimg; b < B; b++) out.counts[b] = -1;
    if (np == 0) return;
    const size_t es = R.bf16 ? 2 : 4;
    RMaps m{};
    for (int l = 0; l < 4; l++) {
        m.p[l] = P[l].p;
        m.h[l] = P[l].h;
        m.w[l] = P[l].w;
    }
    m.C = 256;
    void* maps = R.ar.get(260, (size_t)np * 12544 * es);
    launch_roi_align(m, d_props, d_pimg, np, -1, 0.f, R.bf16, maps, st);
    void* f1 = R.ar.get(261, (size_t)np * 1024 * es);
    void* f2 = R.ar.get(262, (size_t)np * 1024 * es);
    float* ho = R.ar.get<float>(263, (size_t)np * 6);
    cunit(R, R.i_fc, maps, (int)np, 1, 1, f1, 1024, true);
    cunit(R, R.i_fc + 1, f1, (int)np, 1, 1, f2, 1024, true);
    cunit(R, R.i_fc + 2, f2, (int)np, 1, 1, ho, 6, false, nullptr, 0, false, true);
    float4* bx = R.ar.get<float4>(264, np);
    float* sc = R.ar.get<float>(265, np);
    int32_t* fl = R.ar.get<int32_t>(266, np);
    int32_t* inc = R.ar.get<int32_t>(267, np);
    k_roi_post<<<cdiv(np, 256), 256, 0, st>>>(ho, d_props, np, (float)wu, (float)hu, bx, sc, fl);
    inclusive_scan_i32(R.ar, 268, fl, inc, np, st);
    std::vector<int32_t> hf(np);
    VTF_HIP(hipMemcpyAsync(hf.data(), fl, np * 4, hipMemcpyDeviceToHost, st));
    VTF_HIP(hipStreamSynchronize(st));
    int64_t n = 0;
    std::vector<int64_t> calls(B, 0);
    for (int64_t t = 0; t < np; t++)
        if (hf[t]) {
            calls[(int)R.last_props[t * 5]]++;
            n++;
        }
    if (n == 0) return;
    float4* cb = R.ar.get<float4>(269, n);
    float* cs = R.ar.get<float>(270, n);
    int32_t* ci = R.ar.get<int32_t>(271, n);
    k_compact4<int32_t><<<cdiv(np, 256), 256, 0, st>>>(fl, inc, np, bx, sc, d_pimg, cb, cs, ci);
    int32_t* cls = R.ar.get<int32_t>(272, n);
    VTF_HIP(hipMemsetAsync(cls, 0, n * 4, st));
    int32_t* keep = R.ar.get<int32_t>(273, n);
    std::vector<int64_t> nk;
    // final_nms: one batched_nms(0.5) per image, classes all 0 (post.py:4-10)
    nms_multi(R.ar, (const float*)cb, cs, cls, ci, calls, 1, 0.5, keep, nk, st);
    std::vector<int64_t> offs(3 * (size_t)B);
    int64_t kb = 0, ob = 0;
    for (int b = 0; b < B; b++) {
        offs[3 * b] = kb;
        offs[3 * b + 1] = std::min<int64_t>(nk[b], R_FINAL);
        offs[3 * b + 2] = ob;
        if (out.counts[b] >= 0) out.counts[b] = (int32_t)offs[3 * b + 1];
        kb += nk[b];
        ob += offs[3 * b + 1];
    }
    int64_t* doffs = R.ar.get<int64_t>(274, 3 * (size_t)B);
    VTF_HIP(hipMemcpyAsync(doffs, offs.data(), offs.size() * 8, hipMemcpyHostToDevice, st));
    float* drows = R.ar.get<float>(275, std::max<int64_t>(ob, 1) * 5);
    // scale_boxes: torch.tensor(sz_orig) / torch.tensor(sz_used) in fp32, flipped to (x, y)
    const float sx = (float)W / (float)wu, sy = (float)H / (float)hu;
    k_rcnn_final<<<B, 128, 0, st>>>(keep, doffs, cb, cs, sx, sy, R_FINAL, drows);
    out.d_rows = drows;
    out.n = ob;
    if (!out.host) return;
    out.rows.resize((size_t)ob * 5);
    if (ob) VTF_HIP(hipMemcpyAsync(out.rows.data(), drows, ob * 20, hipMemcpyDeviceToHost, st));
    VTF_HIP(hipStreamSynchronize(st));
}

static void heads_alloc(Rcnn& R, int B, int Hp, int Wp, RMap P[R_LEVELS], float* heads[R_LEVELS]) {
    int h = Hp / 4, w = Wp / 4;
    for (int l = 0; l < R_LEVELS; l++) {
        heads[l] = R.ar.get<float>(280 + l, (size_t)B * h * w * 15);
        (void)P;
        h = (h - 1) / 2 + 1;
        w = (w - 1) / 2 + 1;
    }
}

static void detect(Rcnn& R, const uint8_t* frames, int on_dev, int B, int H, int W, int64_t fstride, int64_t rstride,
                   ROut& out) {
    VTF_CHECK(B > 0 && H > 0 && W > 0, VTF_E_ARG, "rcnn: bad shape");
    hipStream_t st = R.st;
    const uint8_t* fr = frames;
    if (!on_dev) {
        uint8_t* d = R.ar.get<uint8_t>(290, (size_t)B * H * W * 3);
        for (int b = 0; b < B; b++)
            VTF_HIP(hipMemcpy2DAsync(d + (size_t)b * H * W * 3, (size_t)W * 3, frames + b * fstride, rstride,
                                     (size_t)W * 3, H, hipMemcpyHostToDevice, st));
        fr = d;
        fstride = (int64_t)H * W * 3;
        rstride = (int64_t)W * 3;
    }
    int hu, wu;
    used_size(H, W, hu, wu);
    const int Hp = (hu + 31) / 32 * 32, Wp = (wu + 31) / 32 * 32;
    void* x0 = R.ar.get(291, (size_t)B * Hp * Wp * 8 * (R.bf16 ? 2 : 4));
    launch_prep(fr, fstride, rstride, B, H, W, hu, wu, Hp, Wp, R.bf16, x0, st);
    RMap P[R_LEVELS];
    float* heads[R_LEVELS];
    heads_alloc(R, B, Hp, Wp, P, heads);
    net(R, x0, B, Hp, Wp, P, heads);
    float4* props = nullptr;
    int32_t* pimg = nullptr;
    int64_t np = rpn_proposals(R, heads, P, B, hu, wu, &props, &pimg);
    roi_stage(R, P, props, pimg, np, B, H, W, hu, wu, out);
}

}  // namespace vtf

using namespace vtf;

struct vtf_rcnn_s {
    Rcnn r;
};

extern "C" {

int vtf_rcnn_create(const float* params, int64_t n_params, int device, int precision, vtf_rcnn_t* out) {
    return guarded([&] {
        VTF_CHECK(params && out && (precision == 0 || precision == 1), VTF_E_ARG, "bad argument");
        DeviceGuard dg(device);
        auto* h = new vtf_rcnn_s();
        h->r.device = device;
        h->r.bf16 = precision == 1;
        try {
            build(h->r, params, n_params);
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
    });
}

int vtf_rcnn_destroy(vtf_rcnn_t h) {
    return guarded_on(h ? h->r.device : -1, [&] { delete h; });
}

int vtf_rcnn_set_stream(vtf_rcnn_t h, void* stream) {
    return guarded_on(h ? h->r.device : -1, [&] {
        VTF_CHECK(h, VTF_E_ARG, "null handle");
        h->r.st = (hipStream_t)stream;
    });
}

int vtf_rcnn_detect_crops(vtf_rcnn_t h, const uint8_t* frames, int frames_on_device, int B, int H, int W,
                          int64_t frame_stride, int64_t row_stride, const vtf_box_params* params,
                          int32_t frame_offset, int32_t* d_crops, int32_t* out_frame_counts, int64_t cap,
                          int64_t* out_n) {
    return guarded_on(h ? h->r.device : -1, [&] {
        VTF_CHECK(h && frames && params && out_n, VTF_E_ARG, "null argument");
        ROut r;
        r.host = false;
        detect(h->r, frames, frames_on_device, B, H, W, frame_stride, row_stride, r);
        VTF_CHECK(r.n == 0 || d_crops, VTF_E_ARG, "null argument");
        rows_to_crops(h->r.ar, 300, r.d_rows, r.counts, H, W, *params, frame_offset, d_crops, nullptr,
                      out_frame_counts, cap, out_n, h->r.st);
    });
}

int vtf_rcnn_input_size(int H, int W, int* out4) {
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

int vtf_rcnn_detect(vtf_rcnn_t h, const uint8_t* frames, int frames_on_device, int B, int H, int W,
                    int64_t frame_stride, int64_t row_stride, float* out_boxes, float* out_scores, int32_t* out_counts,
                    int64_t cap, int64_t* out_total) {
    return guarded_on(h ? h->r.device : -1, [&] {
        VTF_CHECK(h && frames && out_counts, VTF_E_ARG, "null argument");
        ROut r;
        detect(h->r, frames, frames_on_device, B, H, W, frame_stride, row_stride, r);
        int64_t n = (int64_t)r.rows.size() / 5;
        if (out_total) *out_total = n;
        VTF_CHECK(n <= cap, VTF_E_CAPACITY, "output capacity too small");
        for (int b = 0; b < B; b++) out_counts[b] = r.counts[b];
        for (int64_t e = 0; e < n; e++) {
            if (out_boxes) std::memcpy(out_boxes + e * 4, &r.rows[e * 5], 16);
            if (out_scores) out_scores[e] = r.rows[e * 5 + 4];
        }
    });
}

int vtf_rcnn_preprocess(vtf_rcnn_t h, const uint8_t* d_frames, int B, int H, int W, int64_t frame_stride,
                        int64_t row_stride, float* d_out) {
    return guarded_on(h ? h->r.device : -1, [&] {
        VTF_CHECK(h && d_frames && d_out && B > 0, VTF_E_ARG, "bad argument");
        int hu, wu;
        used_size(H, W, hu, wu);
        launch_prep(d_frames, frame_stride, row_stride, B, H, W, hu, wu, (hu + 31) / 32 * 32, (wu + 31) / 32 * 32,
                    false, d_out, h->r.st);
        VTF_HIP(hipStreamSynchronize(h->r.st));
    });
}

int vtf_rcnn_rpn_heads(vtf_rcnn_t h, const float* d_x, int B, int Hp, int Wp, float* d_head0, float* d_head1,
                       float* d_head2, float* d_head3, float* d_head4) {
    return guarded_on(h ? h->r.device : -1, [&] {
        VTF_CHECK(h && d_x && d_head0 && d_head1 && d_head2 && d_head3 && d_head4 && B > 0, VTF_E_ARG, "bad argument");
        Rcnn& R = h->r;
        void* x0 = R.ar.get(291, (size_t)B * Hp * Wp * 8 * (R.bf16 ? 2 : 4));
        launch_nchw_to_nhwc(d_x, B, 3, Hp, Wp, 8, x0, R.bf16, R.st);
        RMap P[R_LEVELS];
        float* heads[R_LEVELS] = {d_head0, d_head1, d_head2, d_head3, d_head4};
        net(R, x0, B, Hp, Wp, P, heads);
        VTF_HIP(hipStreamSynchronize(R.st));
    });
}

int vtf_rcnn_proposals(vtf_rcnn_t h, float* out, int64_t cap, int64_t* out_n) {
    return guarded_on(h ? h->r.device : -1, [&] {
        VTF_CHECK(h && out_n, VTF_E_ARG, "null argument");
        int64_t n = (int64_t)h->r.last_props.size() / 5;
        *out_n = n;
        VTF_CHECK(n <= cap, VTF_E_CAPACITY, "output capacity too small");
        if (n) std::memcpy(out, h->r.last_props.data(), n * 20);
    });
}

int vtf_rcnn_rpn_proposals(vtf_rcnn_t h, const float* d_head0, const float* d_head1, const float* d_head2,
                           const float* d_head3, const float* d_head4, int B, int Hp, int Wp, int h_used, int w_used,
                           float* out, int64_t cap, int64_t* out_n) {
    return guarded_on(h ? h->r.device : -1, [&] {
        VTF_CHECK(h && d_head0 && d_head1 && d_head2 && d_head3 && d_head4 && out_n && B > 0, VTF_E_ARG,
                  "bad argument");
        VTF_CHECK(Hp % 32 == 0 && Wp % 32 == 0 && h_used > 0 && w_used > 0 && h_used <= Hp && w_used <= Wp,
                  VTF_E_ARG, "rcnn: bad input size");
        float* heads[R_LEVELS] = {(float*)d_head0, (float*)d_head1, (float*)d_head2, (float*)d_head3,
                                  (float*)d_head4};
        RMap P[R_LEVELS];
        int hh = Hp / 4, ww = Wp / 4;
        for (int l = 0; l < R_LEVELS; l++) {
            P[l] = RMap{nullptr, hh, ww};
            hh = (hh - 1) / 2 + 1;
            ww = (ww - 1) / 2 + 1;
        }
        float4* props = nullptr;
        int32_t* pimg = nullptr;
        rpn_proposals(h->r, heads, P, B, h_used, w_used, &props, &pimg);
        int64_t n = (int64_t)h->r.last_props.size() / 5;
        *out_n = n;
        VTF_CHECK(n <= cap, VTF_E_CAPACITY, "output capacity too small");
        if (n) std::memcpy(out, h->r.last_props.data(), n * 20);
    });
}

int vtf_roi_align(const float* d_fmap, int N, int H, int W, int C, const float* d_rois, int64_t R, float spatial_scale,
                  float* d_out, void* hip_stream) {
    return guarded([&] {
        VTF_CHECK(d_fmap && d_rois && d_out && N > 0 && H > 0 && W > 0 && C > 0 && R >= 0, VTF_E_ARG, "bad argument");
        if (R == 0) return;
        hipStream_t st = (hipStream_t)hip_stream;
        // rois [R,5] (image, x1, y1, x2, y2) -> float4 boxes + int32 image
        std::vector<float> hr(R * 5);
        VTF_HIP(hipMemcpyAsync(hr.data(), d_rois, R * 20, hipMemcpyDeviceToHost, st));
        VTF_HIP(hipStreamSynchronize(st));
        std::vector<float4> bx(R);
        std::vector<int32_t> im(R);
        for (int64_t r = 0; r < R; r++) {
            im[r] = (int32_t)hr[r * 5];
            VTF_CHECK(im[r] >= 0 && im[r] < N, VTF_E_ARG, "roi_align: image index out of range");
            bx[r] = make_float4(hr[r * 5 + 1], hr[r * 5 + 2], hr[r * 5 + 3], hr[r * 5 + 4]);
        }
        float4* db = nullptr;
        int32_t* di = nullptr;
        VTF_HIP(hipMallocAsync((void**)&db, R * 16, st));
        VTF_HIP(hipMallocAsync((void**)&di, R * 4, st));
        VTF_HIP(hipMemcpyAsync(db, bx.data(), R * 16, hipMemcpyHostToDevice, st));
        VTF_HIP(hipMemcpyAsync(di, im.data(), R * 4, hipMemcpyHostToDevice, st));
        RMaps m{};
        m.p[0] = d_fmap;
        m.h[0] = H;
        m.w[0] = W;
        m.C = C;
        launch_roi_align(m, db, di, R, 0, spatial_scale, false, d_out, st);
        VTF_HIP(hipFreeAsync(db, st));
        VTF_HIP(hipFreeAsync(di, st));
        VTF_HIP(hipStreamSynchronize(st));
    });
}

int vtf_rcnn_profile(vtf_rcnn_t h, int enable, double* out_ms, int64_t* out_launches, double* out_flops,
                     int64_t* out_frames) {
    return guarded_on(h ? h->r.device : -1, [&] {
        VTF_CHECK(h, VTF_E_ARG, "null handle");
        Rcnn& R = h->r;
        if (out_ms) *out_ms = R.prof_ms;
        if (out_launches) *out_launches = R.prof_launches;
        if (out_flops) *out_flops = R.prof_flops;
        if (out_frames) *out_frames = R.prof_frames;
        R.prof_ms = R.prof_flops = 0;
        R.prof_launches = R.prof_frames = 0;
        if (enable) {
            if (!R.ev0) VTF_HIP(hipEventCreate(&R.ev0));
            if (!R.ev1) VTF_HIP(hipEventCreate(&R.ev1));
        }
        R.prof = enable != 0;
    });
}

}  // extern "C"

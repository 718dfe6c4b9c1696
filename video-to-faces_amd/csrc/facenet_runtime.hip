// FaceNet (InceptionResnetV1) runtime: layer table, buffer plan, forward.
// Mirrors src/videotofaces/encoders/facenet.py:10-183 layer for layer; every conv is one
// launch of the implicit-GEMM kernel (conv.hip) with its BN/bias/residual/ReLU epilogue
// fused; concatenations are written in place as channel slices.  Sibling 1x1 convs that read the
// same input (the first conv of every Inception branch) run as one merged launch whose output
// channels are split between the concat buffer and the branch temporaries.
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "blob.hpp"
#include "boxes.hpp"
#include "common.hpp"
#include "conv.hpp"

namespace vtf {

void launch_block17_fused(const void* x, void* y, int N, const void* wm, const float* alm, const float* bem,
                          const void* wa, const float* ala, const float* bea, const void* wb, const float* alb,
                          const float* beb, const void* wo, const float* bo, float scale, hipStream_t st,
                          bool head_only, int ws, int wos);

void launch_block35_branches(const void* x, void* cat, int N, const void* wm, const float* alm, const float* bem,
                             const void* w1, const float* al1, const float* be1, const void* w2a, const float* al2a,
                             const float* be2a, const void* w2b, const float* al2b, const float* be2b,
                             hipStream_t st);

bool launch_conv_patch(const ConvParams& q, hipStream_t st);

void launch_stem_head(const uint8_t* frames, int F, int H, int W, int64_t fstride, int64_t rstride,
                      const int32_t* d_crops, int N, const void* w, const float* al, const float* be, void* out,
                      hipStream_t st);

void launch_block8_mid(const void* t1, void* cat, int N, const void* wa, const float* ala, const float* bea,
                       const void* wb, const float* alb, const float* beb, hipStream_t st, int ws);

// device crops of uint8 frames (vtf_facenet_encode_crops): the bf16 fused mode runs the blob and
// conv2d_1a as one launch (k_stem_head)
struct StemIn {
    const uint8_t* frames;
    int F, H, W;
    int64_t fstride, rstride;
    const int32_t* crops;
};

// bf16 Block17 as one launch per block (facenet_fused.hip); VTF_FN_FUSED=0: the four launches
static bool fused_blocks() {
    const char* e = std::getenv("VTF_FN_FUSED");  // (read per forward: tests switch it in-process)
    return !(e && std::atoi(e) == 0);
}
// Block17 stage 4 (1x1 256 -> 896 + residual) inside the per-image launch (default since round 6:
// with its weights at a padded stride the per-image stream costs less than the batch launch --
// solo forward equal, c2 +0.8 %, profiles/r06_b17_split_c2_ab.txt) or as its own GEMM launch
// over the batch (VTF_B17_SPLIT=1)
static bool b17_split() {
    const char* e = std::getenv("VTF_B17_SPLIT");
    return e && std::atoi(e) != 0;
}

struct Layer {
    int cin, cout, kh, kw, sh, sw, ph, pw;
    bool bias;       // conv2d with bias (block tail) instead of ConvUnit (BN + ReLU)
    int cin_pad;
    void* w;         // [cout][kh*kw*cin_pad], element = precision
    // (bf16) the same rows at a padded stride of ws elements, for the fused Block17 / Block8
    // kernels that stream weights straight into registers (pad_rows)
    void* wp = nullptr;
    int ws = 0;
    float* b;        // bias
    float* alpha;    // BN
    float* beta;
};

struct Facenet {
    int device = 0;
    bool bf16 = false;
    hipStream_t st = 0;
    std::vector<Layer> L;
    // merged sibling 1x1 convs, keyed by their first member's layer index
    std::vector<std::pair<int, Layer>> LM;
    float* head_w = nullptr;  // [512][1792] fp32
    float* head_alpha = nullptr;
    float* head_beta = nullptr;
    std::vector<void*> allocs;
    Arena ar;
    ~Facenet() {
        for (void* p : allocs) (void)hipFree(p);
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

// geometry of every conv in reference state_dict order (specs.py facenet_spec)
struct G {
    int cin, cout, kh, kw, sh, sw, ph, pw;
    bool bias;
};

// Row stride (elements) for the weights the fused bf16 blocks stream from L2 into registers: their
// load instructions read 16 rows x 64 B, and with K * 2 a multiple of 128 B every row's piece sits
// at the same offset of its cache line -- Block17 ran ~25 % slower that way (FaceNet forward
// 1.888 -> 1.800 ms per 128 faces at K + 112, bit-identical, scripts/r06_b17ws.py).
// VTF_FN_WPAD: the pad in elements (multiple of 8; 0 = dense rows)
static int fused_wpad() {
    const char* e = std::getenv("VTF_FN_WPAD");
    const int v = e ? std::atoi(e) : 112;
    return v > 0 && v % 8 == 0 && v <= 128 ? v : 0;
}

static void pad_rows(Facenet& F, Layer& l, int rows, int K) {
    const int pad = fused_wpad();
    l.wp = l.w;
    l.ws = K;
    if (!pad) return;
    const int ws = K + pad;
    void* d = nullptr;
    VTF_HIP(hipMalloc(&d, (size_t)rows * ws * 2 + 16));
    F.allocs.push_back(d);
    VTF_HIP(hipMemset(d, 0, (size_t)rows * ws * 2 + 16));
    VTF_HIP(hipMemcpy2D(d, (size_t)ws * 2, l.w, (size_t)K * 2, (size_t)K * 2, rows, hipMemcpyDeviceToDevice));
    l.wp = d;
    l.ws = ws;
}

static std::vector<G> facenet_geometry() {
    std::vector<G> g = {{3, 32, 3, 3, 2, 2, 0, 0, 0},    {32, 32, 3, 3, 1, 1, 0, 0, 0},
                        {32, 64, 3, 3, 1, 1, 1, 1, 0},   {64, 80, 1, 1, 1, 1, 0, 0, 0},
                        {80, 192, 3, 3, 1, 1, 0, 0, 0},  {192, 256, 3, 3, 2, 2, 0, 0, 0}};
    for (int b = 0; b < 5; b++) {  // Block35
        g.push_back({256, 32, 1, 1, 1, 1, 0, 0, 0});
        g.push_back({256, 32, 1, 1, 1, 1, 0, 0, 0});
        g.push_back({32, 32, 3, 3, 1, 1, 1, 1, 0});
        g.push_back({256, 32, 1, 1, 1, 1, 0, 0, 0});
        g.push_back({32, 32, 3, 3, 1, 1, 1, 1, 0});
        g.push_back({32, 32, 3, 3, 1, 1, 1, 1, 0});
        g.push_back({96, 256, 1, 1, 1, 1, 0, 0, 1});
    }
    g.push_back({256, 384, 3, 3, 2, 2, 0, 0, 0});  // Mixed_6a
    g.push_back({256, 192, 1, 1, 1, 1, 0, 0, 0});
    g.push_back({192, 192, 3, 3, 1, 1, 1, 1, 0});
    g.push_back({192, 256, 3, 3, 2, 2, 0, 0, 0});
    for (int b = 0; b < 10; b++) {  // Block17
        g.push_back({896, 128, 1, 1, 1, 1, 0, 0, 0});
        g.push_back({896, 128, 1, 1, 1, 1, 0, 0, 0});
        g.push_back({128, 128, 1, 7, 1, 1, 0, 3, 0});
        g.push_back({128, 128, 7, 1, 1, 1, 3, 0, 0});
        g.push_back({256, 896, 1, 1, 1, 1, 0, 0, 1});
    }
    g.push_back({896, 256, 1, 1, 1, 1, 0, 0, 0});  // Mixed_7a
    g.push_back({256, 384, 3, 3, 2, 2, 0, 0, 0});
    g.push_back({896, 256, 1, 1, 1, 1, 0, 0, 0});
    g.push_back({256, 256, 3, 3, 2, 2, 0, 0, 0});
    g.push_back({896, 256, 1, 1, 1, 1, 0, 0, 0});
    g.push_back({256, 256, 3, 3, 1, 1, 1, 1, 0});
    g.push_back({256, 256, 3, 3, 2, 2, 0, 0, 0});
    for (int b = 0; b < 6; b++) {  // 5 x Block8 + Block8(relu=False)
        g.push_back({1792, 192, 1, 1, 1, 1, 0, 0, 0});
        g.push_back({1792, 192, 1, 1, 1, 1, 0, 0, 0});
        g.push_back({192, 192, 1, 3, 1, 1, 0, 1, 0});
        g.push_back({192, 192, 3, 1, 1, 1, 1, 0, 0});
        g.push_back({384, 1792, 1, 1, 1, 1, 0, 0, 1});
    }
    return g;
}

static void bn_fold(const float* w, const float* b, const float* mean, const float* var, int n, float eps,
                    std::vector<float>& alpha, std::vector<float>& beta) {
    alpha.resize(n);
    beta.resize(n);
    for (int i = 0; i < n; i++) {
        alpha[i] = w[i] / std::sqrt(var[i] + eps);
        beta[i] = b[i] - mean[i] * alpha[i];
    }
}


static void build(Facenet& F, const float* params, int64_t n_params) {
    std::vector<G> geo = facenet_geometry();
    int64_t src = 0;
    auto take = [&](int64_t n) {
        VTF_CHECK(src + n <= n_params, VTF_E_ARG, "facenet: parameter buffer too small");
        const float* p = params + src;
        src += n;
        return p;
    };
    std::vector<std::vector<float>> host_w;  // per layer [cout][K] fp32 (merged-layer source)
    std::vector<std::vector<float>> host_a, host_b;
    for (const G& g : geo) {
        Layer l{};
        l.cin = g.cin;
        l.cout = g.cout;
        l.kh = g.kh;
        l.kw = g.kw;
        l.sh = g.sh;
        l.sw = g.sw;
        l.ph = g.ph;
        l.pw = g.pw;
        l.bias = g.bias;
        l.cin_pad = (g.cin + 7) / 8 * 8;
        const float* w = take((int64_t)g.cout * g.cin * g.kh * g.kw);
        int K = g.kh * g.kw * l.cin_pad;
        std::vector<float> wt((size_t)g.cout * K, 0.f);
        for (int co = 0; co < g.cout; co++)
            for (int ci = 0; ci < g.cin; ci++)
                for (int y = 0; y < g.kh; y++)
                    for (int x = 0; x < g.kw; x++)
                        wt[(size_t)co * K + (y * g.kw + x) * l.cin_pad + ci] =
                            w[(((size_t)co * g.cin + ci) * g.kh + y) * g.kw + x];
        if (F.bf16) {
            std::vector<uint16_t> wb(wt.size());
            for (size_t i = 0; i < wt.size(); i++) wb[i] = f2bf(wt[i]);
            l.w = F.upload(wb);
        } else {
            l.w = F.upload(wt);
        }
        host_w.push_back(std::move(wt));
        if (g.bias) {
            const float* b = take(g.cout);
            l.b = F.upload(std::vector<float>(b, b + g.cout));
        } else {
            const float* bw = take(g.cout);
            const float* bb = take(g.cout);
            const float* bm = take(g.cout);
            const float* bv = take(g.cout);
            std::vector<float> a, be;
            bn_fold(bw, bb, bm, bv, g.cout, 1e-3f, a, be);  // conv_unit BN eps 1e-3 (facenet.py:11)
            l.alpha = F.upload(a);
            l.beta = F.upload(be);
            host_a.resize(F.L.size() + 1);
            host_b.resize(F.L.size() + 1);
            host_a[F.L.size()] = a;
            host_b[F.L.size()] = be;
        }
        F.L.push_back(l);
    }
    // merged sibling 1x1 convs (same input, BN + ReLU units): weights / BN rows concatenated, so
    // every output channel's dot product and epilogue are those of its own conv
    auto merge = [&](std::vector<int> ids) {
        Layer m = F.L[ids[0]];
        std::vector<float> w, a, be;
        m.cout = 0;
        for (int i : ids) {
            VTF_CHECK(F.L[i].kh == 1 && F.L[i].kw == 1 && F.L[i].cin == m.cin && !F.L[i].bias, VTF_E_ARG,
                      "facenet: merged convs must be sibling 1x1 units");
            w.insert(w.end(), host_w[i].begin(), host_w[i].end());
            a.insert(a.end(), host_a[i].begin(), host_a[i].end());
            be.insert(be.end(), host_b[i].begin(), host_b[i].end());
            m.cout += F.L[i].cout;
        }
        if (F.bf16) {
            std::vector<uint16_t> wb(w.size());
            for (size_t i = 0; i < w.size(); i++) wb[i] = f2bf(w[i]);
            m.w = F.upload(wb);
        } else {
            m.w = F.upload(w);
        }
        m.alpha = F.upload(a);
        m.beta = F.upload(be);
        F.LM.push_back({ids[0], m});
    };
    for (int k = 0; k < 5; k++) merge({6 + 7 * k, 7 + 7 * k, 9 + 7 * k});  // Block35 branches 0, 1, 2
    for (int k = 0; k < 10; k++) merge({45 + 5 * k, 46 + 5 * k});         // Block17 branches 0, 1
    merge({95, 97, 99});                                                   // Mixed_7a branches 0, 1, 2
    for (int k = 0; k < 6; k++) merge({102 + 5 * k, 103 + 5 * k});        // Block8 branches 0, 1
    if (F.bf16) {
        // padded-stride copies for the fused Block17 (merged head 896 -> 256, 1x7, 7x1) and Block8
        // middle (1x3, 3x1) kernels
        for (int k = 0; k < 10; k++) {
            for (auto& e : F.LM)
                if (e.first == 45 + 5 * k) pad_rows(F, e.second, 256, 896);
            pad_rows(F, F.L[47 + 5 * k], 128, 896);
            pad_rows(F, F.L[48 + 5 * k], 128, 896);
            pad_rows(F, F.L[49 + 5 * k], 896, 256);  // the 1x1 256 -> 896 (stage 4 in the per-image form)
        }
        for (int k = 0; k < 6; k++) {
            pad_rows(F, F.L[104 + 5 * k], 192, 576);
            pad_rows(F, F.L[105 + 5 * k], 192, 576);
        }
    }
    const float* hw = take(512 * 1792);
    F.head_w = F.upload(std::vector<float>(hw, hw + 512 * 1792));
    const float* bw = take(512);
    const float* bb = take(512);
    const float* bm = take(512);
    const float* bv = take(512);
    std::vector<float> a, be;
    bn_fold(bw, bb, bm, bv, 512, 1e-3f, a, be);  // BatchNorm1d(512, 0.001) (facenet.py:147)
    F.head_alpha = F.upload(a);
    F.head_beta = F.upload(be);
    VTF_CHECK(src == n_params, VTF_E_ARG, "facenet: expected 23512224 parameters");
}

struct Act {
    void* p;
    int H, W, C;
};

// in_cstride / in_coff: read channels [in_coff, in_coff + in.C) of a buffer with in_cstride
// channels per pixel (0: the input is dense)
static void conv(Facenet& F, int li, const Act& in, int N, void* out, int out_cstride, int out_coff,
                 const void* res = nullptr, float scale = 1.f, bool relu = true, Act* out_act = nullptr,
                 int in_cstride = 0, int in_coff = 0) {
    const Layer& l = F.L[li];
    VTF_CHECK(in.C == l.cin_pad, VTF_E_ARG, "facenet: channel mismatch");
    ConvParams p{};
    p.in = (const char*)in.p + (size_t)in_coff * (F.bf16 ? 2 : 4);
    p.in_cstride = in_cstride;
    p.w = l.w;
    p.out = out;
    p.N = N;
    p.H = in.H;
    p.W = in.W;
    p.Cin = l.cin_pad;
    p.KH = l.kh;
    p.KW = l.kw;
    p.sh = l.sh;
    p.sw = l.sw;
    p.ph = l.ph;
    p.pw = l.pw;
    p.OH = (in.H + 2 * l.ph - l.kh) / l.sh + 1;
    p.OW = (in.W + 2 * l.pw - l.kw) / l.sw + 1;
    p.Cout = l.cout;
    p.K = l.kh * l.kw * l.cin_pad;
    p.M = (int64_t)N * p.OH * p.OW;
    p.out_cstride = out_cstride;
    p.out_coff = out_coff;
    if (l.bias) {
        p.bias = l.b;
        p.scale = scale;
        p.res = res;
        p.res_cstride = l.cout;
        p.relu = relu;
    } else {
        p.alpha = l.alpha;
        p.beta = l.beta;
        p.scale = 1.f;
        p.relu = 1;
    }
    // the stem's 3x3 stride-1 convs on 32 channels: patch convs in the fused bf16 mode
    if (!(F.bf16 && fused_blocks() && launch_conv_patch(p, F.st))) launch_conv(p, F.bf16, F.st);
    if (out_act) *out_act = Act{out, p.OH, p.OW, out_cstride};
}

// merged sibling 1x1 convs whose first member is layer li: output channels [0, n_split) to
// out (out_cstride, out_coff), the rest to out2 (out2_cstride, out2_coff)
static void conv_merged(Facenet& F, int li, const Act& in, int N, void* out, int out_cstride, int out_coff,
                        int n_split, void* out2, int out2_cstride, int out2_coff) {
    const Layer* l = nullptr;
    for (auto& e : F.LM)
        if (e.first == li) l = &e.second;
    VTF_CHECK(l && in.C == l->cin_pad, VTF_E_ARG, "facenet: no merged conv at this layer");
    ConvParams p{};
    p.in = in.p;
    p.w = l->w;
    p.out = out;
    p.N = N;
    p.H = in.H;
    p.W = in.W;
    p.Cin = l->cin_pad;
    p.KH = p.KW = p.sh = p.sw = 1;
    p.OH = in.H;
    p.OW = in.W;
    p.Cout = l->cout;
    p.K = l->cin_pad;
    p.M = (int64_t)N * p.OH * p.OW;
    p.out_cstride = out_cstride;
    p.out_coff = out_coff;
    p.alpha = l->alpha;
    p.beta = l->beta;
    p.scale = 1.f;
    p.relu = 1;
    p.n_split = n_split;
    p.out2 = out2;
    p.out2_cstride = out2_cstride;
    p.out2_coff = out2_coff;
    launch_conv(p, F.bf16, F.st);
}

// x: NHWC [N,160,160,8] (precision dtype) -> emb [N,512] fp32; or (stem) the crops, blob and
// conv2d_1a fused
static void forward(Facenet& F, const void* x, int N, float* emb, const StemIn* stem = nullptr) {
    const size_t es = F.bf16 ? 2 : 4;
    const size_t big = (size_t)N * 77 * 77 * 64;  // largest activation (stem conv2)
    const size_t tmp = (size_t)N * 17 * 17 * 192;  // largest branch temp (Mixed_6a)
    const size_t cat = (size_t)N * 17 * 17 * 96;
    void* P0 = F.ar.get(0, big * es);
    void* P1 = F.ar.get(1, big * es);
    void* T1 = F.ar.get(2, tmp * es);
    void* T2 = F.ar.get(3, tmp * es);
    void* CAT = F.ar.get(4, cat * es);
    Act a{(void*)x, 160, 160, 8}, b{};
    int li = 0;
    // stem (facenet.py:126-134)
    if (stem) {
        const Layer& l0 = F.L[0];
        VTF_CHECK(F.bf16 && l0.cin_pad == 8 && l0.cout == 32 && l0.kh == 3 && l0.kw == 3 && l0.sh == 2 && l0.sw == 2 &&
                      l0.ph == 0 && l0.pw == 0 && !l0.bias,
                  VTF_E_ARG, "facenet: stem head shape");
        launch_stem_head(stem->frames, stem->F, stem->H, stem->W, stem->fstride, stem->rstride, stem->crops, N, l0.w,
                         l0.alpha, l0.beta, P0, F.st);
        b = Act{P0, 79, 79, 32};
        li++;
    } else {
        conv(F, li++, a, N, P0, 32, 0, nullptr, 1.f, true, &b);
    }
    conv(F, li++, b, N, P1, 32, 0, nullptr, 1.f, true, &a);
    conv(F, li++, a, N, P0, 64, 0, nullptr, 1.f, true, &b);
    launch_maxpool(P0, N, b.H, b.W, 64, P1, 64, 0, F.bf16, F.st);
    a = Act{P1, (b.H - 3) / 2 + 1, (b.W - 3) / 2 + 1, 64};
    conv(F, li++, a, N, P0, 80, 0, nullptr, 1.f, true, &b);
    conv(F, li++, b, N, P1, 192, 0, nullptr, 1.f, true, &a);
    conv(F, li++, a, N, P0, 256, 0, nullptr, 1.f, true, &b);
    Act X = b;
    void* Y = P1;
    auto swap = [&](int C) {
        void* old = X.p;
        X.p = Y;
        X.C = C;
        Y = old;
    };
    Act t1{}, t2{};
    // 5 x Block35 (facenet.py:14-33), scale 0.17
    for (int k = 0; k < 5; k++) {
        if (F.bf16 && fused_blocks() && X.H == 17 && X.W == 17 && X.C == 256) {
            // the three branches in one launch into CAT, then the tail conv
            const Layer* lm = nullptr;
            for (auto& e : F.LM)
                if (e.first == li) lm = &e.second;
            VTF_CHECK(lm, VTF_E_ARG, "facenet: no merged Block35 head");
            const Layer &l1 = F.L[li + 2], &l2a = F.L[li + 4], &l2b = F.L[li + 5];
            launch_block35_branches(X.p, CAT, N, lm->w, lm->alpha, lm->beta, l1.w, l1.alpha, l1.beta, l2a.w, l2a.alpha,
                                    l2a.beta, l2b.w, l2b.alpha, l2b.beta, F.st);
            li += 6;
            conv(F, li++, Act{CAT, X.H, X.W, 96}, N, Y, 256, 0, X.p, 0.17f, true);
            swap(256);
            continue;
        }
        // branch 0 -> CAT[0:32]; branch 1 / 2 heads -> T1[0:32] / T1[32:64]
        conv_merged(F, li, X, N, CAT, 96, 0, 32, T1, 64, 0);
        li += 2;
        conv(F, li++, Act{T1, X.H, X.W, 32}, N, CAT, 96, 32, nullptr, 1.f, true, nullptr, 64, 0);
        li++;
        conv(F, li++, Act{T1, X.H, X.W, 32}, N, T2, 32, 0, nullptr, 1.f, true, &t2, 64, 32);
        conv(F, li++, t2, N, CAT, 96, 64);
        conv(F, li++, Act{CAT, X.H, X.W, 96}, N, Y, 256, 0, X.p, 0.17f, true);
        swap(256);
    }
    // Mixed_6a (facenet.py:84-101)
    {
        Act o{};
        conv(F, li++, X, N, Y, 896, 0, nullptr, 1.f, true, &o);
        conv(F, li++, X, N, T1, 192, 0, nullptr, 1.f, true, &t1);
        conv(F, li++, t1, N, T2, 192, 0, nullptr, 1.f, true, &t2);
        conv(F, li++, t2, N, Y, 896, 384);
        launch_maxpool(X.p, N, X.H, X.W, 256, Y, 896, 640, F.bf16, F.st);
        X.H = o.H;
        X.W = o.W;
        swap(896);
    }
    // 10 x Block17 (facenet.py:36-56), scale 0.10
    for (int k = 0; k < 10; k++) {
        if (F.bf16 && fused_blocks() && X.H == 8 && X.W == 8 && X.C == 896) {
            const Layer* lm = nullptr;
            for (auto& e : F.LM)
                if (e.first == li) lm = &e.second;
            VTF_CHECK(lm, VTF_E_ARG, "facenet: no merged Block17 head");
            const Layer &la = F.L[li + 2], &lb = F.L[li + 3], &lo = F.L[li + 4];
            const bool split = b17_split();
            VTF_CHECK(lm->wp && la.wp && lb.wp && lo.wp && lm->ws == la.ws && la.ws == lb.ws, VTF_E_ARG,
                      "facenet: Block17 padded weights");
            launch_block17_fused(X.p, split ? CAT : Y, N, lm->wp, lm->alpha, lm->beta, la.wp, la.alpha, la.beta, lb.wp,
                                 lb.alpha, lb.beta, lo.wp, lo.b, 0.10f, F.st, split, la.ws, lo.ws);
            li += 4;
            if (split)  // the tail: the unfused path's conv (same k order and epilogue)
                conv(F, li, Act{CAT, X.H, X.W, 256}, N, Y, 896, 0, X.p, 0.10f, true);
            li++;
            swap(896);
            continue;
        }
        conv_merged(F, li, X, N, CAT, 256, 0, 128, T1, 128, 0);
        li += 2;
        t1 = Act{T1, X.H, X.W, 128};
        conv(F, li++, t1, N, T2, 128, 0, nullptr, 1.f, true, &t2);
        conv(F, li++, t2, N, CAT, 256, 128);
        conv(F, li++, Act{CAT, X.H, X.W, 256}, N, Y, 896, 0, X.p, 0.10f, true);
        swap(896);
    }
    // Mixed_7a (facenet.py:104-120)
    {
        Act o{};
        // the three branch heads (1x1, 896 -> 256 each) as one launch into T1 [.., 768]
        conv_merged(F, li, X, N, T1, 768, 0, 0, nullptr, 0, 0);
        const Act h{T1, X.H, X.W, 256};
        li++;
        conv(F, li++, h, N, Y, 1792, 0, nullptr, 1.f, true, &o, 768, 0);
        li++;
        conv(F, li++, h, N, Y, 1792, 384, nullptr, 1.f, true, nullptr, 768, 256);
        li++;
        conv(F, li++, h, N, T2, 256, 0, nullptr, 1.f, true, &t2, 768, 512);
        conv(F, li++, t2, N, Y, 1792, 640);
        launch_maxpool(X.p, N, X.H, X.W, 896, Y, 1792, 896, F.bf16, F.st);
        X.H = o.H;
        X.W = o.W;
        swap(1792);
    }
    // 5 x Block8 (scale 0.20) + Block8(scale 1.0, relu=False) (facenet.py:59-81,142-143)
    for (int k = 0; k < 6; k++) {
        bool last = k == 5;
        conv_merged(F, li, X, N, CAT, 384, 0, 192, T1, 192, 0);
        li += 2;
        const char* b8e = std::getenv("VTF_B8_MID");  // 0: the two launches (A/B; read per forward)
        if (F.bf16 && fused_blocks() && !(b8e && std::atoi(b8e) == 0) && X.H == 3 && X.W == 3 && X.C == 1792) {
            // the branch's 1x3 and 3x1 convs as one launch (facenet_fused.hip)
            const Layer &la = F.L[li], &lb = F.L[li + 1];
            VTF_CHECK(la.cin_pad == 192 && la.cout == 192 && la.kh == 1 && la.kw == 3 && la.pw == 1 && lb.cin_pad == 192 &&
                          lb.cout == 192 && lb.kh == 3 && lb.kw == 1 && lb.ph == 1,
                      VTF_E_ARG, "facenet: Block8 middle shape");
            VTF_CHECK(la.wp && lb.wp && la.ws == lb.ws, VTF_E_ARG, "facenet: Block8 padded weights");
            launch_block8_mid(T1, CAT, N, la.wp, la.alpha, la.beta, lb.wp, lb.alpha, lb.beta, F.st, la.ws);
            li += 2;
        } else {
            t1 = Act{T1, X.H, X.W, 192};
            conv(F, li++, t1, N, T2, 192, 0, nullptr, 1.f, true, &t2);
            conv(F, li++, t2, N, CAT, 384, 192);
        }
        conv(F, li++, Act{CAT, X.H, X.W, 384}, N, Y, 1792, 0, X.p, last ? 1.0f : 0.20f, !last);
        swap(1792);
    }
    VTF_CHECK(li == (int)F.L.size(), VTF_E_ARG, "facenet: layer walk mismatch");
    // AdaptiveAvgPool2d(1) + Linear + BatchNorm1d + F.normalize (facenet.py:144-153)
    float* hs = F.ar.get<float>(7, (size_t)N * (1792 + 512));
    launch_facenet_head(X.p, N, X.H * X.W, 1792, F.head_w, F.head_alpha, F.head_beta, 512, emb, hs, F.bf16, F.st);
}

}  // namespace vtf

using namespace vtf;

struct vtf_facenet_s {
    Facenet f;
};

extern "C" {

int vtf_facenet_create(const float* params, int64_t n_params, int device, int precision, vtf_facenet_t* out) {
    return guarded([&] {
        VTF_CHECK(params && out && (precision == 0 || precision == 1), VTF_E_ARG, "bad argument");
        DeviceGuard dg(device);
        auto* h = new vtf_facenet_s();
        h->f.device = device;
        h->f.bf16 = precision == 1;
        try {
            build(h->f, params, n_params);
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
    });
}

int vtf_facenet_destroy(vtf_facenet_t h) {
    return guarded_on(h ? h->f.device : -1, [&] { delete h; });
}

int vtf_facenet_set_stream(vtf_facenet_t h, void* stream) {
    return guarded_on(h ? h->f.device : -1, [&] {
        VTF_CHECK(h, VTF_E_ARG, "null handle");
        h->f.st = (hipStream_t)stream;
    });
}

int vtf_facenet_forward(vtf_facenet_t h, const float* d_x, int64_t N, float* d_emb) {
    return guarded_on(h ? h->f.device : -1, [&] {
        VTF_CHECK(h && N >= 0, VTF_E_ARG, "bad argument");
        if (N == 0) return;
        VTF_CHECK(d_x && d_emb, VTF_E_ARG, "null argument");
        Facenet& F = h->f;
        void* xin = F.ar.get(5, (size_t)N * 160 * 160 * 8 * (F.bf16 ? 2 : 4));
        launch_nchw_to_nhwc(d_x, (int)N, 3, 160, 160, 8, xin, F.bf16, F.st);
        forward(F, xin, (int)N, d_emb);
        VTF_HIP(hipGetLastError());
    });
}

int vtf_facenet_encode_crops(vtf_facenet_t h, const uint8_t* d_frames, int n_frames, int H, int W,
                             int64_t frame_stride, int64_t row_stride, const int32_t* crops, int crops_on_device,
                             int64_t N, float* d_emb) {
    return guarded_on(h ? h->f.device : -1, [&] {
        VTF_CHECK(h && N >= 0 && n_frames > 0 && H > 0 && W > 0, VTF_E_ARG, "bad argument");
        if (N == 0) return;
        VTF_CHECK(d_frames && crops && d_emb, VTF_E_ARG, "null argument");
        Facenet& F = h->f;
        const int32_t* dc = crops;
        if (!crops_on_device) {
            check_crops_host(crops, N, n_frames, H, W);
            int32_t* d = F.ar.get<int32_t>(6, N * 5);
            VTF_HIP(hipMemcpyAsync(d, crops, N * 5 * 4, hipMemcpyHostToDevice, F.st));
            dc = d;
        }
        if (F.bf16 && fused_blocks()) {
            const StemIn si{d_frames, n_frames, H, W, frame_stride, row_stride, dc};
            forward(F, nullptr, (int)N, d_emb, &si);
            VTF_HIP(hipGetLastError());
            return;
        }
        void* xin = F.ar.get(5, (size_t)N * 160 * 160 * 8 * (F.bf16 ? 2 : 4));
        // blobFromImages(images, 1/128, (160,160), (127.5,)*3, swapRB=True) (facenet.py:179)
        launch_blob(d_frames, n_frames, H, W, frame_stride, row_stride, dc, N, 160, 127.5f, 0.0078125f, 1, 8, F.bf16, xin, F.st);
        forward(F, xin, (int)N, d_emb);
        VTF_HIP(hipGetLastError());
    });
}

}  // extern "C"

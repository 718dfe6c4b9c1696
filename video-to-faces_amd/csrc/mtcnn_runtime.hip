// MTCNN detector runtime: weights, pyramid plan, stage orchestration (host side).
// Mirrors MTCNN.forward (src/videotofaces/detectors/mtcnn.py:167-252) step by step; every
// data-dependent size is read back once per stage (detect(): 1 + 3 NMS + 2 compaction syncs, the
// final rows left pending for the caller's one sync).
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <numeric>
#include <vector>

#include "boxes.hpp"
#include "common.hpp"
#include "conv.hpp"
#include "gemm_x3.hpp"
#include "mtcnn.hpp"
#include "nms.hpp"

namespace vtf {

__global__ void k_iota(int32_t* v, int64_t n) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) v[i] = (int32_t)i;
}
__global__ void k_desc_keys(const float* s, int64_t n, uint64_t* k) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) k[i] = desc_key(s[i]);
}
// Final rows grouped by image, keeping the IoM keep order inside each image (the reference
// splits the kept boxes per image with boolean masks, mtcnn.py:244-249): row k of the keep list
// is element order[pos[k]].  One workgroup: a stable counting sort by image (per-image counts,
// their exclusive scan, then each 1024-row chunk ranks its rows among equal images).
__global__ __launch_bounds__(1024) void k_mtcnn_rows(const int32_t* __restrict__ order, const int32_t* __restrict__ pos,
                                                     const int32_t* __restrict__ d_nf, const int32_t* __restrict__ img,
                                                     const float4* __restrict__ box, const float* __restrict__ score,
                                                     const float* __restrict__ lm, int B, float* __restrict__ rows,
                                                     float* __restrict__ lmo, int32_t* __restrict__ counts,
                                                     int32_t* __restrict__ mail) {
    __shared__ int s_cnt[4096];
    __shared__ int s_base[4096];
    __shared__ int s_img[1024];
    const int tid = threadIdx.x;
    const int nf = *d_nf;  // kept rows (the IoM compaction's inclusive count)
    if (tid == 0) mail[0] = nf;
    for (int b = tid; b < B; b += 1024) s_cnt[b] = 0;
    __syncthreads();
    for (int k = tid; k < nf; k += 1024) atomicAdd(&s_cnt[img[order[pos[k]]]], 1);
    __syncthreads();
    if (tid == 0) {
        int acc = 0;
        for (int b = 0; b < B; b++) {
            s_base[b] = acc;
            counts[b] = s_cnt[b];
            mail[1 + b] = s_cnt[b];
            acc += s_cnt[b];
            s_cnt[b] = 0;
        }
    }
    __syncthreads();
    for (int c0 = 0; c0 < nf; c0 += 1024) {
        const int k = c0 + tid;
        int e = -1, b = -1;
        if (k < nf) {
            e = order[pos[k]];
            b = img[e];
        }
        s_img[tid] = b;
        __syncthreads();
        if (k < nf) {
            int rank = 0;
            for (int j = 0; j < tid; j++) rank += s_img[j] == b;
            const int dst = s_base[b] + s_cnt[b] + rank;
            const float4 bx = box[e];
            float* o = rows + (int64_t)dst * 5;
            o[0] = bx.x;
            o[1] = bx.y;
            o[2] = bx.z;
            o[3] = bx.w;
            o[4] = score[e];
            for (int j = 0; j < 10; j++) lmo[(int64_t)dst * 10 + j] = lm[(int64_t)e * 10 + j];
        }
        __syncthreads();
        if (k < nf) atomicAdd(&s_cnt[b], 1);
        __syncthreads();
    }
}

__global__ void k_gather_order(const int32_t* order, const int32_t* pos, int64_t n, int64_t* out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) out[i] = order[pos[i]];
}
__global__ void k_gather_rows(const int32_t* idx, int64_t n, const float* in, int row, float* out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n * row) return;
    int64_t k = i / row;
    int j = (int)(i % row);
    out[i] = in[(int64_t)idx[k] * row + j];
}

struct Mtcnn {
    int device = 0;
    int sat_pk = 0;  // the current det-batch's SAT layout (mtcnn_dev.hpp; launch_sat)
    hipStream_t st = 0;
    float* d_w = nullptr;
    PNetW pw{};
    // RNet / ONet as conv-kernel layers (fp32, [Cout_p][KH][KW][Cin_p]) + heads
    struct CL {
        int cin, cout, k;
        const float *w, *b, *a;
        const void* sp;  // the weights in the split-pair layout (conv_dma split mode), or null
    };
    std::vector<CL> rl, ol;
    const float* fw[2] = {nullptr, nullptr};  // conv1 of RNet / ONet for k_cand_front: [28][32]
    const float *rh1w, *rh1b, *rh2w, *rh2b;                    // rnet dense5_1 / dense5_2
    const float *oh1w, *oh1b, *oh2w, *oh2b, *oh3w, *oh3b;      // onet dense6_1 / 6_2 / 6_3
    Arena ar;
    int64_t stats[8] = {0};
    // parity introspection (vtf_mtcnn_stage1_keys): the last call's stage-1 candidate keys
    bool keep_s1 = false;
    std::vector<uint64_t> s1_keys;
    // kernel timing (vtf_mtcnn_profile)
    bool prof = false;
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    double prof_ms = 0, prof_flops = 0;
    int64_t prof_launches = 0, prof_frames = 0;

    std::vector<void*> allocs;
    // RNet / ONet convs: 0 fp32 MFMA; 1 split-fp16 conv mode, operand range proven from the
    // weights; 2 split-fp16 guarded: a device flag reports an operand >= 2^14 and the net re-runs
    // in fp32
    int cand_x[2] = {0, 0};
    // stage control words: [0] conv-layer guard, [1] fused front-half guard, [2] out-of-frame
    // candidate counter (err), [3] spare; zeroed by the gather launch that opens each stage
    int* d_ovf = nullptr;
    // level plan last uploaded to S_LVC (re-uploaded only when it changes)
    std::vector<PNetLevel> lv_host;
    const PNetLevel* lv_dev = nullptr;
    // fused RNet / ONet front half (mtcnn_cand.hip); used when the split mode is allowed
    CandFusedW cf[2]{};
    bool fused = false;
    // RNet / ONet on the LDS-DMA conv kernel's split mode with split-pair activations
    // (VTF_MTCNN_SP=0: k_conv's staging-split mode)
    bool sp = true;
    // VTF_PNET_PRIO=1: k_pnet on a lowest-priority stream of this handle (the other lanes' stage-2/3
    // and encoder kernels are dispatched ahead of its workgroups); joined back by events
    hipStream_t pst = nullptr;
    hipEvent_t pev[2] = {nullptr, nullptr};
    ~Mtcnn() {
        if (pst) (void)hipStreamDestroy(pst);
        for (hipEvent_t e : pev)
            if (e) (void)hipEventDestroy(e);
        for (void* p : allocs) (void)hipFree(p);
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        if (d_w) (void)hipFree(d_w);
        if (d_ovf) (void)hipFree(d_ovf);
    }
};

enum Slot {
    S_FRAMES = 0, S_LEVELS, S_COUNT, S_KEY, S_SCORE, S_REGV, S_KEY2, S_SLOT, S_SLOT2, S_B1, S_S1, S_R1, S_I1, S_C1,
    S_KEEP, S_B2, S_S2, S_R2, S_I2, S_C2, S_PROB, S_REG, S_LM, S_ERR, S_FLAG, S_INCL, S_IDX, S_LMK, S_OUTB, S_OUTS,
    S_OUTL, S_OUTI, S_SORT, S_SCAN, S_PRE, S_CROP, S_SAT, S_LVC, S_VR
};
static_assert(S_VR < 40, "nms_multi owns arena slots 40-63");
// host mailboxes (Arena::mail): stage-1 counts, stage-2/3 compaction results, final rows, box post
enum MailSlot { M_COUNT = 0, M_STAGE = 1, M_ROWS = 2, M_BOXES = 3 };

// ---- weights: reference state_dict order (specs.py mtcnn_spec) -> transposed device layout
static void build_weights(Mtcnn& m, const float* params, int64_t n_params) {
    struct P {
        const char* name;
        int co, ci, kh, kw;  // conv: co,ci,kh,kw; dense: co=out, ci=in, kh=kw=0; vec: co=n, ci=0
        int kind;            // 0 vec, 1 conv (transpose), 2 dense (keep [out][in]), 3 dense transposed,
                             // 4 conv kept [co][ci][kh][kw] (PNet conv1: per-channel rows for scalar loads)
    };
    static const P spec[] = {
        {"pnet.conv1.w", 10, 3, 3, 3, 4},   {"pnet.conv1.b", 10, 0, 0, 0, 0},   {"pnet.prelu1", 10, 0, 0, 0, 0},
        {"pnet.conv2.w", 16, 10, 3, 3, 1},  {"pnet.conv2.b", 16, 0, 0, 0, 0},   {"pnet.prelu2", 16, 0, 0, 0, 0},
        {"pnet.conv3.w", 32, 16, 3, 3, 1},  {"pnet.conv3.b", 32, 0, 0, 0, 0},   {"pnet.prelu3", 32, 0, 0, 0, 0},
        {"pnet.conv4_1.w", 2, 32, 0, 0, 2}, {"pnet.conv4_1.b", 2, 0, 0, 0, 0},  {"pnet.conv4_2.w", 4, 32, 0, 0, 2},
        {"pnet.conv4_2.b", 4, 0, 0, 0, 0},
        {"rnet.conv1.w", 28, 3, 3, 3, 1},   {"rnet.conv1.b", 28, 0, 0, 0, 0},   {"rnet.prelu1", 28, 0, 0, 0, 0},
        {"rnet.conv2.w", 48, 28, 3, 3, 1},  {"rnet.conv2.b", 48, 0, 0, 0, 0},   {"rnet.prelu2", 48, 0, 0, 0, 0},
        {"rnet.conv3.w", 64, 48, 2, 2, 1},  {"rnet.conv3.b", 64, 0, 0, 0, 0},   {"rnet.prelu3", 64, 0, 0, 0, 0},
        {"rnet.dense4.w", 128, 576, 0, 0, 3}, {"rnet.dense4.b", 128, 0, 0, 0, 0}, {"rnet.prelu4", 128, 0, 0, 0, 0},
        {"rnet.dense5_1.w", 2, 128, 0, 0, 2}, {"rnet.dense5_1.b", 2, 0, 0, 0, 0}, {"rnet.dense5_2.w", 4, 128, 0, 0, 2},
        {"rnet.dense5_2.b", 4, 0, 0, 0, 0},
        {"onet.conv1.w", 32, 3, 3, 3, 1},   {"onet.conv1.b", 32, 0, 0, 0, 0},   {"onet.prelu1", 32, 0, 0, 0, 0},
        {"onet.conv2.w", 64, 32, 3, 3, 1},  {"onet.conv2.b", 64, 0, 0, 0, 0},   {"onet.prelu2", 64, 0, 0, 0, 0},
        {"onet.conv3.w", 64, 64, 3, 3, 1},  {"onet.conv3.b", 64, 0, 0, 0, 0},   {"onet.prelu3", 64, 0, 0, 0, 0},
        {"onet.conv4.w", 128, 64, 2, 2, 1}, {"onet.conv4.b", 128, 0, 0, 0, 0},  {"onet.prelu4", 128, 0, 0, 0, 0},
        {"onet.dense5.w", 256, 1152, 0, 0, 3}, {"onet.dense5.b", 256, 0, 0, 0, 0}, {"onet.prelu5", 256, 0, 0, 0, 0},
        {"onet.dense6_1.w", 2, 256, 0, 0, 2}, {"onet.dense6_1.b", 2, 0, 0, 0, 0}, {"onet.dense6_2.w", 4, 256, 0, 0, 2},
        {"onet.dense6_2.b", 4, 0, 0, 0, 0}, {"onet.dense6_3.w", 10, 256, 0, 0, 2}, {"onet.dense6_3.b", 10, 0, 0, 0, 0},
    };
    const int NP = sizeof(spec) / sizeof(spec[0]);
    std::vector<float> host;
    std::vector<int64_t> off(NP);
    int64_t src = 0;
    for (int i = 0; i < NP; i++) {
        const P& p = spec[i];
        int64_t n = (p.kind == 0) ? p.co : (p.kind == 1 || p.kind == 4 ? (int64_t)p.co * p.ci * p.kh * p.kw : (int64_t)p.co * p.ci);
        VTF_CHECK(src + n <= n_params, VTF_E_ARG, "mtcnn: parameter buffer too small");
        off[i] = (int64_t)host.size();
        const float* s = params + src;
        if (p.kind == 1) {
            int K = p.ci * p.kh * p.kw;
            for (int k = 0; k < K; k++)
                for (int co = 0; co < p.co; co++) host.push_back(s[(int64_t)co * K + k]);
        } else if (p.kind == 3) {
            for (int k = 0; k < p.ci; k++)
                for (int co = 0; co < p.co; co++) host.push_back(s[(int64_t)co * p.ci + k]);
        } else {  // kinds 0, 2, 4: reference layout
            host.insert(host.end(), s, s + n);
        }
        while (host.size() % 4) host.push_back(0.f);  // 16-B alignment for every tensor
        src += n;
    }
    VTF_CHECK(src == n_params, VTF_E_ARG, "mtcnn: expected 495850 parameters");
    VTF_HIP(hipMalloc(&m.d_w, host.size() * 4));
    VTF_HIP(hipMemcpy(m.d_w, host.data(), host.size() * 4, hipMemcpyHostToDevice));
    {
        const float* b = m.d_w;
        int i = 0;
        auto nx = [&]() { return b + off[i++]; };
        m.pw = PNetW{nx(), nx(), nx(), nx(), nx(), nx(), nx(), nx(), nx(), nx(), nx(), nx(), nx(), nullptr, nullptr, nullptr, nullptr, 0};
    }
    // raw (reference layout) tensors by spec index
    std::vector<const float*> raw(NP);
    {
        int64_t o = 0;
        for (int i = 0; i < NP; i++) {
            const P& p = spec[i];
            raw[i] = params + o;
            o += (p.kind == 0) ? p.co : (p.kind == 1 || p.kind == 4 ? (int64_t)p.co * p.ci * p.kh * p.kw : (int64_t)p.co * p.ci);
        }
    }
    // conv-kernel layers: weights [Cout_p][kh][kw][Cin_p], zero padded; bias, prelu padded.
    // flat=true: a dense layer over a [3,3,C] map whose reference flatten order is
    // permute(0,3,2,1) -> (w, h, c) (mtcnn.py:68,113); the conv kernel's k order is (h, w, c).
    auto layer = [&](int wi, int cin, int cin_p, int cout, int k, bool flat) {
        int cout_p = (cout + 7) / 8 * 8;
        std::vector<float> w((size_t)cout_p * k * k * cin_p, 0.f), b(cout_p, 0.f), a(cout_p, 0.f);
        const float* W = raw[wi];
        for (int co = 0; co < cout; co++)
            for (int y = 0; y < k; y++)
                for (int x = 0; x < k; x++)
                    for (int ci = 0; ci < cin; ci++) {
                        float v = flat ? W[(size_t)co * (k * k * cin) + (x * k + y) * cin + ci]
                                       : W[(((size_t)co * cin + ci) * k + y) * k + x];
                        w[(((size_t)co * k + y) * k + x) * cin_p + ci] = v;
                    }
        for (int co = 0; co < cout; co++) {
            b[co] = raw[wi + 1][co];
            a[co] = raw[wi + 2][co];
        }
        Mtcnn::CL L{cin_p, cout_p, k, nullptr, nullptr, nullptr, nullptr};
        if (k * k * cin_p % 8 == 0) {
            std::vector<uint16_t> h((size_t)cout_p * k * k * cin_p * 2);
            if (split_rows_host(w.data(), cout_p, k * k * cin_p, h.data())) {
                void* d = nullptr;
                VTF_HIP(hipMalloc(&d, h.size() * 2));
                VTF_HIP(hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice));
                m.allocs.push_back(d);
                L.sp = d;
            }
        }
        float* d = nullptr;
        VTF_HIP(hipMalloc(&d, (w.size() + b.size() + a.size()) * 4));
        VTF_HIP(hipMemcpy(d, w.data(), w.size() * 4, hipMemcpyHostToDevice));
        VTF_HIP(hipMemcpy(d + w.size(), b.data(), b.size() * 4, hipMemcpyHostToDevice));
        VTF_HIP(hipMemcpy(d + w.size() + b.size(), a.data(), a.size() * 4, hipMemcpyHostToDevice));
        m.allocs.push_back(d);
        L.w = d;
        L.b = d + w.size();
        L.a = d + w.size() + b.size();
        return L;
    };
    // spec indices: rnet.conv1.w = 13 ... (see the table above)
    m.rl = {layer(13, 3, 8, 28, 3, false), layer(16, 28, 32, 48, 3, false), layer(19, 48, 48, 64, 2, false),
            layer(22, 64, 64, 128, 3, true)};
    m.ol = {layer(29, 3, 8, 32, 3, false),  layer(32, 32, 32, 64, 3, false), layer(35, 64, 64, 64, 3, false),
            layer(38, 64, 64, 128, 2, false), layer(41, 128, 128, 256, 3, true)};
    // conv1 of RNet / ONet as [k = (c, ky, kx)][co] (k = 27 and co >= Cout zero) for the
    // fused candidate front end (k_cand_front)
    for (int net = 0; net < 2; net++) {
        const int wi = net ? 29 : 13, cout = net ? 32 : 28;
        std::vector<float> w(28 * 32, 0.f);
        for (int co = 0; co < cout; co++)
            for (int kk = 0; kk < 27; kk++) w[kk * 32 + co] = raw[wi][(size_t)co * 27 + kk];
        float* d = nullptr;
        VTF_HIP(hipMalloc(&d, w.size() * 4));
        VTF_HIP(hipMemcpy(d, w.data(), w.size() * 4, hipMemcpyHostToDevice));
        m.allocs.push_back(d);
        m.fw[net] = d;
    }
    // PNet conv3 on the fp16 matrix cores (k_pnet): x = x0 + x1 * 2^-11 and w = w0 + w1 * 2^-11
    // with fp16 parts represent both operands to ~2^-24 relative and x*w = x0 w0 + 2^-11 (x0 w1 +
    // x1 w0) drops only x1 w1 (<= 2^-24 relative): fp32-grade products.  The conv2 activations
    // must stay inside the fp16 range: bound them from the weights (level inputs lie in
    // [-1, 1]); beyond the bound k_pnet keeps the fp32 MFMA path.
    // operand bound of a conv / dense layer with PReLU: max_co (sum_k |w| * in + |b|) * max(1, |slope|)
    auto bound = [&](int wi, int co, int K, double in) {
        const float* W = raw[wi];
        double b = 0.0, amax = 1.0;
        for (int c = 0; c < co; c++) {
            double s = std::fabs((double)raw[wi + 1][c]);
            for (int k = 0; k < K; k++) s += std::fabs((double)W[(size_t)c * K + k]) * in;
            b = std::max(b, s);
            amax = std::max(amax, std::fabs((double)raw[wi + 2][c]));
        }
        return b * amax;
    };
    const char* force = std::getenv("VTF_MTCNN_FP32");  // tests: force the fp32 MFMA paths
    const bool allow_x = !(force && force[0] == '1');
    // RNet / ONet layers on the conv kernel's split-fp16 mode when every operand stays < 2^14
    {
        const double r1 = bound(13, 28, 27, 1.0), r2 = bound(16, 48, 28 * 9, r1), r3 = bound(19, 64, 48 * 4, r2);
        m.cand_x[0] = !allow_x ? 0 : (r1 < 16384.0 && r2 < 16384.0 && r3 < 16384.0 ? 1 : 2);
        const double o1 = bound(29, 32, 27, 1.0), o2 = bound(32, 64, 32 * 9, o1), o3 = bound(35, 64, 64 * 9, o2),
                     o4 = bound(38, 128, 64 * 4, o3);
        m.cand_x[1] = !allow_x ? 0 : (o1 < 16384.0 && o2 < 16384.0 && o3 < 16384.0 && o4 < 16384.0 ? 1 : 2);
        VTF_HIP(hipMalloc((void**)&m.d_ovf, 16));
        // the fused front half is opt-in (VTF_MTCNN_FUSED=1): correct (tests/test_mtcnn_gpu.py) but
        // measured slower than the layer path on MI355X (ONet 347 vs ~300 ns per candidate chip-wide,
        // RNet 93 vs ~80; profiles/r02b_probe_cand.txt): at 137 KB of LDS one workgroup per CU
        // cannot hide its own barrier / LDS latency
        const char* fz = std::getenv("VTF_MTCNN_FUSED");
        m.fused = fz && fz[0] == '1';
        const char* spe = std::getenv("VTF_MTCNN_SP");
        m.sp = !(spe && spe[0] == '0');
        // split fp16 planes of conv1 ([2][32][64], k = ky*16 + kx*4 + c) and conv2 ([2][C2][288],
        // k = tap*32 + ci) for the fused front half
        auto split_to = [&](std::vector<uint16_t>& h, size_t i0, size_t i1, float w) {
            const _Float16 w0 = (_Float16)w;
            const _Float16 w1 = (_Float16)((w - (float)w0) * 2048.f);
            std::memcpy(&h[i0], &w0, 2);
            std::memcpy(&h[i1], &w1, 2);
        };
        auto upload = [&](const std::vector<uint16_t>& h) {
            uint16_t* d = nullptr;
            VTF_HIP(hipMalloc((void**)&d, h.size() * 2));
            VTF_HIP(hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice));
            m.allocs.push_back((void*)d);
            return (const _Float16*)d;
        };
        for (int net = 0; net < 2; net++) {
            const int wc1 = net ? 29 : 13, wc2 = net ? 32 : 16;
            const int co1 = net ? 32 : 28, ci2 = co1, co2 = net ? 64 : 48;
            std::vector<uint16_t> h1((size_t)2 * 32 * 64, 0), h2((size_t)2 * co2 * 288, 0);
            for (int co = 0; co < co1; co++)
                for (int c = 0; c < 3; c++)
                    for (int ky = 0; ky < 3; ky++)
                        for (int kx = 0; kx < 3; kx++)
                            split_to(h1, (size_t)co * 64 + ky * 16 + kx * 4 + c, (size_t)(32 + co) * 64 + ky * 16 + kx * 4 + c,
                                     raw[wc1][((co * 3 + c) * 3 + ky) * 3 + kx]);
            for (int co = 0; co < co2; co++)
                for (int ci = 0; ci < ci2; ci++)
                    for (int t = 0; t < 9; t++)
                        split_to(h2, (size_t)co * 288 + t * 32 + ci, (size_t)(co2 + co) * 288 + t * 32 + ci,
                                 raw[wc2][((size_t)co * ci2 + ci) * 9 + t]);
            const auto& L = net ? m.ol : m.rl;
            m.cf[net] = CandFusedW{upload(h1), L[0].b, L[0].a, upload(h2), L[1].b, L[1].a};
        }
    }
    {
        const double b1 = bound(0, 10, 27, 1.0), b2 = bound(3, 16, 90, b1);
        if (b1 < 16384.0 && b2 < 16384.0 && allow_x) {
            // [2][co][144] split planes of a [co][ci][3][3] conv, k = tap * 16 + ci
            auto split = [&](const float* W, int co_n, int ci_n) {
                std::vector<uint16_t> h((size_t)2 * co_n * 144, 0);
                for (int co = 0; co < co_n; co++)
                    for (int tap = 0; tap < 9; tap++)
                        for (int ci = 0; ci < ci_n; ci++) {
                            const float w = W[((size_t)co * ci_n + ci) * 9 + tap];
                            const _Float16 w0 = (_Float16)w;
                            const _Float16 w1 = (_Float16)((w - (float)w0) * 2048.f);
                            // rows >= 16: the tap's channel halves swapped (k_pnet C3_SWZ)
                            const int cs = co >= 16 ? ci ^ 8 : ci;
                            std::memcpy(&h[(size_t)co * 144 + tap * 16 + cs], &w0, 2);
                            std::memcpy(&h[(size_t)(co_n + co) * 144 + tap * 16 + cs], &w1, 2);
                        }
                uint16_t* d = nullptr;
                VTF_HIP(hipMalloc((void**)&d, h.size() * 2));
                VTF_HIP(hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice));
                m.allocs.push_back((void*)d);
                return (const uint16_t*)d;
            };
            {
                std::vector<uint16_t> h((size_t)2 * 16 * 64, 0);
                const float* W = raw[0];  // [10][3][3][3]
                for (int co = 0; co < 10; co++)
                    for (int c = 0; c < 3; c++)
                        for (int ky = 0; ky < 3; ky++)
                            for (int kx = 0; kx < 3; kx++) {
                                const float w = W[((co * 3 + c) * 3 + ky) * 3 + kx];
                                const _Float16 w0 = (_Float16)w;
                                const _Float16 w1 = (_Float16)((w - (float)w0) * 2048.f);
                                const int k = ky * 16 + kx * 4 + c;
                                std::memcpy(&h[(size_t)co * 64 + k], &w0, 2);
                                std::memcpy(&h[(size_t)(16 + co) * 64 + k], &w1, 2);
                            }
                uint16_t* d = nullptr;
                VTF_HIP(hipMalloc((void**)&d, h.size() * 2));
                VTF_HIP(hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice));
                m.allocs.push_back((void*)d);
                m.pw.c1h = d;
            }
            {
                // conv2 [2][16][96]: k = 32 s + 8 g + j packs the 90 (tap, ci) products in 3 steps
                // (k_pnet conv2): s < 2 -> tap 4 s + g, ci j; s = 2 -> g 0: tap 8, ci j; g 1 / 2:
                // tap 4 (g - 1) + j / 2, ci 8 + j % 2; g 3: tap 8, ci 8 + j (j < 2), else zero
                std::vector<uint16_t> h((size_t)2 * 16 * 96, 0);
                const float* W = raw[3];  // [16][10][3][3]
                for (int co = 0; co < 16; co++)
                    for (int k = 0; k < 96; k++) {
                        const int st = k / 32, g = (k % 32) / 8, j = k % 8;
                        int tap = -1, ci = -1;
                        if (st < 2) tap = 4 * st + g, ci = j;
                        else if (g == 0) tap = 8, ci = j;
                        else if (g < 3) tap = 4 * (g - 1) + j / 2, ci = 8 + j % 2;
                        else if (j < 2) tap = 8, ci = 8 + j;
                        if (tap < 0) continue;
                        const float w = W[((size_t)co * 10 + ci) * 9 + tap];
                        const _Float16 w0 = (_Float16)w;
                        const _Float16 w1 = (_Float16)((w - (float)w0) * 2048.f);
                        std::memcpy(&h[(size_t)co * 96 + k], &w0, 2);
                        std::memcpy(&h[(size_t)(16 + co) * 96 + k], &w1, 2);
                    }
                uint16_t* d = nullptr;
                VTF_HIP(hipMalloc((void**)&d, h.size() * 2));
                VTF_HIP(hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice));
                m.allocs.push_back((void*)d);
                m.pw.c2h = d;
            }
            m.pw.c3h = split(raw[6], 32, 16);
            if (bound(6, 32, 144, b2) < 16384.0) {  // conv3 activations feed the split heads
                // [2][32 rows][32 k]: k = 16 s + 8 hk + i holds channel 16 s + 8 (i >> 2) + (i & 3)
                // + 4 hk -- the conv3 accumulator register 8 s + i of lane half hk (k_pnet's 32x32
                // conv3); rows 0, 1 conv4_1, 2..5 conv4_2, the rest zero
                std::vector<uint16_t> h(2 * 32 * 32, 0);
                for (int r = 0; r < 6; r++)
                    for (int k = 0; k < 32; k++) {
                        const int s = k >> 4, hk = (k >> 3) & 1, i = k & 7;
                        const int ch = 16 * s + 8 * (i >> 2) + (i & 3) + 4 * hk;
                        const float w = r < 2 ? raw[9][r * 32 + ch] : raw[11][(r - 2) * 32 + ch];
                        const _Float16 w0 = (_Float16)w;
                        const _Float16 w1 = (_Float16)((w - (float)w0) * 2048.f);
                        std::memcpy(&h[(size_t)r * 32 + k], &w0, 2);
                        std::memcpy(&h[(size_t)(32 + r) * 32 + k], &w1, 2);
                    }
                uint16_t* d = nullptr;
                VTF_HIP(hipMalloc((void**)&d, h.size() * 2));
                VTF_HIP(hipMemcpy(d, h.data(), h.size() * 2, hipMemcpyHostToDevice));
                m.allocs.push_back((void*)d);
                m.pw.hh = d;
            }
        }
    }
    {
        auto unit = [&](int idx, int n) {
            for (int c = 0; c < n; c++)
                if (!(raw[idx][c] >= 0.f && raw[idx][c] <= 1.f)) return false;
            return true;
        };
        m.pw.unit_slopes = (unit(5, 16) ? 1 : 0) | (unit(8, 32) ? 2 : 0);  // p2 [16], p3 [32]
        // k_pnet's merged-chain conv1 scales the fp16 w0 plane by 2^11 on the device: exact when
        // every |w| < 16 (2^11 * 16 = 2^15 < 65504)
        bool small = true;
        for (int i = 0; i < 270; i++) small = small && std::fabs(raw[0][i]) < 16.f;
        const char* ck = std::getenv("VTF_PNET_C1K");
        m.pw.c1k = small && !(ck && ck[0] == '0') ? 1 : 0;
    }
    // k_pnet addresses the PNet weights from two bases with constant offsets (mtcnn_kernels.hip
    // PW_* / PH_*): the fp32 tensors are the first 13 of the packed buffer; the fp16 split
    // planes are gathered into one buffer [conv3 | conv2 | conv1 | heads] (zeros where a plane is
    // absent; the kernel only reads a plane when its path is enabled)
    {
        const int64_t want[13] = {0, 272, 284, 296, 1736, 1752, 1768, 6376, 6408, 6440, 6504, 6508, 6636};
        for (int i = 0; i < 13; i++)
            VTF_CHECK(off[i] == want[i], VTF_E_LIMIT, "mtcnn: PNet weight layout differs from k_pnet's offsets");
        if (m.pw.c3h) {
            VTF_CHECK(m.pw.c2h && m.pw.c1h, VTF_E_LIMIT, "mtcnn: split conv3 without split conv1/conv2 planes");
            uint16_t* comb = nullptr;
            VTF_HIP(hipMalloc((void**)&comb, 16384 * 2));
            VTF_HIP(hipMemset(comb, 0, 16384 * 2));
            VTF_HIP(hipMemcpy(comb, m.pw.c3h, 9216 * 2, hipMemcpyDeviceToDevice));
            VTF_HIP(hipMemcpy(comb + 9216, m.pw.c2h, 3072 * 2, hipMemcpyDeviceToDevice));
            VTF_HIP(hipMemcpy(comb + 12288, m.pw.c1h, 2048 * 2, hipMemcpyDeviceToDevice));
            if (m.pw.hh) VTF_HIP(hipMemcpy(comb + 14336, m.pw.hh, 2048 * 2, hipMemcpyDeviceToDevice));
            m.allocs.push_back((void*)comb);
            m.pw.c3h = comb;
            m.pw.c2h = comb + 9216;
            m.pw.c1h = comb + 12288;
            if (m.pw.hh) m.pw.hh = comb + 14336;
        } else {
            m.pw.hh = nullptr;  // the split heads read the conv3 split path's accumulators
        }
    }
    auto dev = [&](int i) { return m.d_w + off[i]; };
    m.rh1w = dev(25); m.rh1b = dev(26); m.rh2w = dev(27); m.rh2b = dev(28);
    m.oh1w = dev(44); m.oh1b = dev(45); m.oh2w = dev(46); m.oh2b = dev(47); m.oh3w = dev(48); m.oh3b = dev(49);
}

// RNet / ONet on NHWC fp32 crops x0 [n,S,S,8] (mtcnn.py:58-76 / 101-121), layer by layer on
// the MFMA conv kernel; pools are torch MaxPool2d(ceil_mode=True).
enum RSlot { S_RA = 70, S_RB = 71, S_BOXPOST = 72, S_CLK = 73 };  // nms_multi owns slots 40-63
// first = 1: x0 is the fused front end's pooled conv1 map [n,P,P,32] (k_cand_front)
static void run_candidates(Mtcnn& m, bool onet, const float* x0, int64_t n, float4* reg, float* lm, float* prob,
                           int first = 0, int force_fp32 = 0) {
    if (n <= 0) return;
    const int xmode = force_fp32 ? 0 : m.cand_x[onet ? 1 : 0];
    if (xmode == 2) VTF_HIP(hipMemsetAsync(m.d_ovf, 0, 4, m.st));
    const int npool_done = first == 2 ? 2 : 0;  // the fused front half ends with pool2
    const int S = onet ? 48 : 24;
    const auto& Ls = onet ? m.ol : m.rl;
    // pools after each conv except the last two of RNet / last two of ONet
    const int pk[5] = {3, 3, onet ? 2 : 0, 0, 0};
    const int npool = onet ? 3 : 2;
    size_t big = (size_t)n * (S - 2) * (S - 2) * 32;
    float* X = m.ar.get<float>(S_RA, big);
    float* Y = m.ar.get<float>(S_RB, big);
    const float* cur = x0;
    int H = S, W = S, C = 8;
    if (first == 1) {
        H = W = cand_front_side(onet);
        C = 32;
    } else if (first == 2) {
        H = W = cand_fused_side(onet);
        C = onet ? 64 : 48;
    }
    for (size_t li = first; li < Ls.size(); li++) {
        const auto& L = Ls[li];
        float* out = (cur == X) ? Y : X;
        ConvParams p{};
        p.in = cur;
        p.w = L.w;
        p.out = out;
        p.bias = L.b;
        p.prelu = L.a;
        p.scale = 1.f;
        p.N = (int)n;
        p.H = H;
        p.W = W;
        p.Cin = C;
        p.KH = p.KW = L.k;
        p.sh = p.sw = 1;
        p.OH = H - L.k + 1;
        p.OW = W - L.k + 1;
        p.Cout = L.cout;
        p.K = L.k * L.k * C;
        p.M = (int64_t)n * p.OH * p.OW;
        p.out_cstride = L.cout;
        p.f16x = xmode != 0;
        p.ovf = xmode == 2 ? m.d_ovf : nullptr;
        // the dense layers run on 120-200 tiles of long K: split-K (slice-order reduction;
        // parity is a tolerance here)
        p.split_fp32 = 1;
        VTF_CHECK(C == L.cin, VTF_E_ARG, "candidate net channel mismatch");
        launch_conv(p, false, m.st);
        H = p.OH;
        W = p.OW;
        C = L.cout;
        cur = out;
        if ((int)li < npool && (int)li >= npool_done) {
            float* pout = (out == X) ? Y : X;
            int OH, OW;
            launch_maxpool_ks(out, (int)n, H, W, C, pk[li], 2, true, pout, OH, OW, m.st);
            H = OH;
            W = OW;
            cur = pout;
        }
    }
    VTF_CHECK(H == 1 && W == 1, VTF_E_ARG, "candidate net shape walk mismatch");
    if (xmode == 2) {  // guarded split-fp16: an out-of-range operand -> the whole net again in fp32
        int ovf = 0;
        VTF_HIP(hipMemcpyAsync(&ovf, m.d_ovf, 4, hipMemcpyDeviceToHost, m.st));
        VTF_HIP(hipStreamSynchronize(m.st));
        if (ovf) {
            run_candidates(m, onet, x0, n, reg, lm, prob, first, 1);
            return;
        }
    }
    if (onet)
        launch_heads(cur, n, C, m.oh1w, m.oh1b, m.oh2w, m.oh2b, m.oh3w, m.oh3b, prob, reg, lm, m.st);
    else
        launch_heads(cur, n, C, m.rh1w, m.rh1b, m.rh2w, m.rh2b, nullptr, nullptr, prob, reg, nullptr, m.st);
}

// RNet / ONet after the candidate front end on the LDS-DMA conv kernel's split mode
// (conv_dma.hip): x0 = k_cand_front's pooled conv1 map [n,P,P,32] in the split-pair layout.  A
// layer feeding a conv writes split pairs from its epilogue, a layer feeding a pool writes fp32
// and the pool writes split pairs; every split-pair producer raises d_ovf[0] on an operand
// beyond the fp16 range (the caller then re-runs the net in fp32).  Same k order and MFMA chains
// as k_conv's split mode.
static void run_candidates_sp(Mtcnn& m, bool onet, const void* x0, int64_t n, float4* reg, float* lm, float* prob) {
    const auto& Ls = onet ? m.ol : m.rl;
    const int pk[5] = {3, 3, onet ? 2 : 0, 0, 0};
    const int npool = onet ? 3 : 2;
    const int S = onet ? 48 : 24;
    size_t big = (size_t)n * (S - 2) * (S - 2) * 32;
    float* X = m.ar.get<float>(S_RA, big);
    float* Y = m.ar.get<float>(S_RB, big);
    const void* cur = x0;
    int H = cand_front_side(onet), W = H, C = 32;
    for (size_t li = 1; li < Ls.size(); li++) {
        const auto& L = Ls[li];
        float* out = (cur == (const void*)X) ? Y : X;
        const bool pool = (int)li < npool;
        const bool last = li + 1 == Ls.size();
        ConvParams p{};
        p.in = cur;
        p.in_sp = 1;
        p.w = L.sp;
        p.out = out;
        p.bias = L.b;
        p.prelu = L.a;
        p.scale = 1.f;
        p.N = (int)n;
        p.H = H;
        p.W = W;
        p.Cin = C;
        p.KH = p.KW = L.k;
        p.sh = p.sw = 1;
        p.OH = H - L.k + 1;
        p.OW = W - L.k + 1;
        p.Cout = L.cout;
        p.K = L.k * L.k * C;
        p.M = (int64_t)n * p.OH * p.OW;
        p.out_cstride = L.cout;
        p.out_sp = !pool && !last;
        p.ovf = m.d_ovf;
        p.split_fp32 = 1;  // slice-order reduction of small grids (parity is a tolerance here)
        VTF_CHECK(C == L.cin && L.sp, VTF_E_ARG, "candidate net channel mismatch");
        if (pool) {
            // conv + pool in one launch when the shape fits (RNet conv2, ONet conv2): the conv
            // map stays in LDS, only the pooled split pairs are written
            float* pout = (out == X) ? Y : X;
            int OH, OW;
            if (launch_conv_span_pool(p, pk[li], 2, pout, OH, OW, m.st)) {
                H = OH;
                W = OW;
                C = L.cout;
                cur = pout;
                continue;
            }
        }
        launch_conv_dma(p, false, m.st);
        H = p.OH;
        W = p.OW;
        C = L.cout;
        cur = out;
        if (pool) {
            float* pout = (out == X) ? Y : X;
            int OH, OW;
            launch_maxpool_ks_sp(out, (int)n, H, W, C, pk[li], 2, true, pout, OH, OW, m.d_ovf, m.st);
            H = OH;
            W = OW;
            cur = pout;
        }
    }
    VTF_CHECK(H == 1 && W == 1, VTF_E_ARG, "candidate net shape walk mismatch");
    const float* f = (const float*)cur;
    if (onet)
        launch_heads(f, n, C, m.oh1w, m.oh1b, m.oh2w, m.oh2b, m.oh3w, m.oh3b, prob, reg, lm, m.st);
    else
        launch_heads(f, n, C, m.rh1w, m.rh1b, m.rh2w, m.rh2b, nullptr, nullptr, prob, reg, nullptr, m.st);
}

// stage 2 / 3 nets on the stage's candidates (mtcnn.py:213-216 / 228-230): the fused front half
// (crop .. pool2 in LDS, split fp16) + the remaining layers batched; on a fused-guard trip
// (an operand beyond the fp16 range) or without the split mode, the layer-by-layer path.
// deferred != null: the caller zeroed d_ovf / err in the stage's opening launch and reads the guard
// back with its compaction sync (*deferred = true when the guarded split path ran); it then calls
// cand_rerun_fp32 if the guard tripped.
static void cand_nets(Mtcnn& m, bool onet, const void* sat, int H, int W, const float4* boxes, const int32_t* img,
                      int64_t n, float4* reg, float* lm, float* prob, int32_t* err, bool* deferred = nullptr) {
    if (n <= 0) return;
    hipStream_t st = m.st;
    const int net = onet ? 1 : 0;
    if (m.fused && m.cand_x[net] != 0) {
        const int P2 = cand_fused_side(onet), C2 = onet ? 64 : 48;
        float* x2 = m.ar.get<float>(S_CROP, (size_t)n * P2 * P2 * C2);
        VTF_HIP(hipMemsetAsync(m.d_ovf + 1, 0, 4, st));
        launch_cand_fused(onet, sat, m.sat_pk, H, W, boxes, img, n, m.cf[net], x2, err, m.d_ovf + 1, st);
        run_candidates(m, onet, x2, n, reg, lm, prob, 2);
        int f_ovf = 0;
        VTF_HIP(hipMemcpyAsync(&f_ovf, m.d_ovf + 1, 4, hipMemcpyDeviceToHost, st));
        VTF_HIP(hipStreamSynchronize(st));
        if (!f_ovf) return;
        VTF_HIP(hipMemsetAsync(err, 0, 4, st));
    }
    const int P = cand_front_side(onet);
    float* x0 = m.ar.get<float>(S_CROP, (size_t)n * P * P * 32);
    const int rl = net;
    bool sp_ok = m.sp && m.cand_x[net] != 0 && !m.fused;
    for (size_t li = 1; li < (onet ? m.ol : m.rl).size(); li++) sp_ok = sp_ok && (onet ? m.ol : m.rl)[li].sp;
    if (sp_ok) {
        // split-pair path: front end writes split pairs, layers on the LDS-DMA conv kernel
        if (!deferred) VTF_HIP(hipMemsetAsync(m.d_ovf, 0, 4, st));
        launch_cand_front(onet, sat, m.sat_pk, H, W, boxes, img, n, m.fw[rl], m.cf[net].w1h, onet ? m.ol[0].b : m.rl[0].b,
                          onet ? m.ol[0].a : m.rl[0].a, x0, err, st, m.d_ovf);
        run_candidates_sp(m, onet, x0, n, reg, lm, prob);
        if (m.cand_x[net] == 1) return;  // operand range proven from the weights
        if (deferred) {
            *deferred = true;
            return;
        }
        int ovf = 0;
        VTF_HIP(hipMemcpyAsync(&ovf, m.d_ovf, 4, hipMemcpyDeviceToHost, st));
        VTF_HIP(hipStreamSynchronize(st));
        if (!ovf) return;
        VTF_HIP(hipMemsetAsync(err, 0, 4, st));  // the fp32 re-run counts invalid boxes again
        launch_cand_front(onet, sat, m.sat_pk, H, W, boxes, img, n, m.fw[rl], nullptr, onet ? m.ol[0].b : m.rl[0].b,
                          onet ? m.ol[0].a : m.rl[0].a, x0, err, st);
        run_candidates(m, onet, x0, n, reg, lm, prob, 1, 1);
        return;
    }
    // conv1 on split fp16 unless the fp32 paths are forced (crop values lie in [-1, 1]: no range
    // guard needed)
    launch_cand_front(onet, sat, m.sat_pk, H, W, boxes, img, n, m.fw[rl], m.cand_x[net] != 0 ? m.cf[net].w1h : nullptr,
                      onet ? m.ol[0].b : m.rl[0].b, onet ? m.ol[0].a : m.rl[0].a, x0, err, st);
    run_candidates(m, onet, x0, n, reg, lm, prob, 1, m.fused && m.cand_x[net] != 0 ? 1 : 0);
}

// MTCNN._scale_pyramid (mtcnn.py:141-148): Python double math, int() truncation
static void plan_levels(int B, int H, int W, double minsize, std::vector<PNetLevel>& lv, int64_t& tiles,
                        int64_t& cells) {
    lv.clear();
    double s = 12.0 / minsize;
    std::vector<double> scales;
    while ((double)std::min(H, W) * s >= 12.0) {
        scales.push_back(s);
        s *= 0.709;
    }
    tiles = 0;
    cells = 0;
    for (double sc : scales) {
        PNetLevel L{};
        L.lh = (int)((double)H * sc + 1.0);
        L.lw = (int)((double)W * sc + 1.0);
        L.ph = (L.lh - 2 + 1) / 2 - 4;
        L.pw = (L.lw - 2 + 1) / 2 - 4;
        L.scale = (float)sc;
        L.tiles_y = cdiv(L.ph, PNET_TH);
        L.tiles_x = cdiv(L.pw, PNET_TW);
        L.tile_beg = tiles;
        // k_pnet's bin math is 32-bit (udiv_est): numerators (lh + 1) H, (lw + 1) W below 2^31
        VTF_CHECK((int64_t)(L.lh + 1) * H < ((int64_t)1 << 31) && (int64_t)(L.lw + 1) * W < ((int64_t)1 << 31),
                  VTF_E_LIMIT, "mtcnn: pyramid level too large for PNet's 32-bit bin math");
        tiles += (int64_t)B * L.tiles_x * L.tiles_y;
        cells += (int64_t)B * L.ph * L.pw;
        lv.push_back(L);
    }
}

// algorithmic FLOPs of PNet per frame over the pyramid (2*MAC; conv1, conv2, conv3, heads)
static double pnet_flops(const std::vector<PNetLevel>& lv) {
    double f = 0;
    for (const PNetLevel& L : lv) {
        double c1 = (double)(L.lh - 2) * (L.lw - 2);
        double p1 = (double)(L.ph + 4) * (L.pw + 4);
        double c2 = (double)(L.ph + 2) * (L.pw + 2);
        double c3 = (double)L.ph * L.pw;
        f += 2.0 * (c1 * 10 * 27 + c2 * 16 * 90 + c3 * 32 * 144 + c3 * 6 * 32);
        (void)p1;
    }
    return f;
}

static void d2h_sync(void* dst, const void* src, size_t bytes, hipStream_t st) {
    VTF_HIP(hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, st));
    VTF_HIP(hipStreamSynchronize(st));
}

// the guarded split path tripped (an operand reached the fp16 range): the stage's nets again on
// the fp32 path (the error counter recounts out-of-frame candidates)
static void cand_rerun_fp32(Mtcnn& m, bool onet, const void* sat, int H, int W, const float4* boxes,
                            const int32_t* img, int64_t n, float4* reg, float* lm, float* prob, int32_t* err) {
    hipStream_t st = m.st;
    const int net = onet ? 1 : 0;
    const int P = cand_front_side(onet);
    float* x0 = m.ar.get<float>(S_CROP, (size_t)n * P * P * 32);
    VTF_HIP(hipMemsetAsync(err, 0, 4, st));
    launch_cand_front(onet, sat, m.sat_pk, H, W, boxes, img, n, m.fw[net], nullptr, onet ? m.ol[0].b : m.rl[0].b,
                      onet ? m.ol[0].a : m.rl[0].a, x0, err, st);
    run_candidates(m, onet, x0, n, reg, lm, prob, 1, 1);
}

// compaction of rows whose score passes `> thr`: returns count, indices in d_idx (order kept).
// The count and the stage's control words (ctl[0] conv guard, [1] fused guard, [2] err) come back
// through the mailbox in the one sync of the stage.
static int64_t threshold_compact(Mtcnn& m, const float* d_s, int64_t n, float thr, int32_t* d_idx, int32_t ctl[3]) {
    ctl[0] = ctl[1] = ctl[2] = 0;
    if (n <= 0) return 0;
    Arena::Mail mb = m.ar.mail(M_STAGE, 16);
    int32_t* flag = m.ar.get<int32_t>(S_FLAG, n);
    int32_t* incl = m.ar.get<int32_t>(S_INCL, n);
    launch_threshold(d_s, n, thr, flag, m.st);
    inclusive_scan_i32(m.ar, S_SCAN, flag, incl, n, m.st);
    launch_flag_compact(flag, incl, n, d_idx, m.st, (int32_t*)mb.d, m.d_ovf, 3);
    VTF_HIP(hipStreamSynchronize(m.st));
    const int32_t* h = (const int32_t*)mb.h;
    ctl[0] = h[1], ctl[1] = h[2], ctl[2] = h[3];
    return h[0];
}

__global__ void k_mail_u32(const uint32_t* __restrict__ src, uint32_t* __restrict__ dst, int n) {
    for (int i = threadIdx.x; i < n; i += blockDim.x) dst[i] = src[i];
}

// final detections in HBM: rows [n,5] (x1,y1,x2,y2,score) and landmarks [n,10] grouped by image
// in the reference's order.  pending: the last stage's launches are queued, not synced -- the
// row count and the per-image counts arrive in `mail` ([0] n, [1 + b] count of image b) at the
// caller's next sync, and d_counts holds the counts in HBM for device consumers (box post).
// Otherwise (an early exit) n and counts are final on the host.
struct DetectOut {
    const float* rows = nullptr;
    const float* lms = nullptr;
    const int32_t* d_counts = nullptr;
    const int32_t* mail = nullptr;
    bool pending = false;
    int64_t n = 0;
    std::vector<int32_t> counts;
    // after the caller's sync: n and counts from the mailbox
    void settle(Mtcnn& m) {
        if (!pending) return;
        pending = false;
        n = mail[0];
        for (size_t b = 0; b < counts.size(); b++) counts[b] = mail[1 + b];
        m.stats[7] = n;
    }
};

// MTCNN.forward (mtcnn.py:167-252) for one det-batch.  Host syncs: the stage-1 candidate count,
// one per batched_nms call (nms_multi), one per stage-2/3 compaction (its count, the stage's
// guard and error words come back together through a mailbox); the final rows are left pending.
// Small host->device tables go through pinned mailboxes and memsets are folded into the stage
// launches, so the det-batch runs no runtime blit copy or fill kernel.
static void detect(Mtcnn& m, const uint8_t* frames, int on_dev, int B, int H, int W, int64_t fstride,
                   int64_t rstride, double minsize, DetectOut& out) {
    VTF_CHECK(B > 0 && H > 0 && W > 0 && minsize > 0, VTF_E_ARG, "mtcnn: bad shape");
    hipStream_t st = m.st;
    std::memset(m.stats, 0, sizeof(m.stats));
    out.rows = out.lms = nullptr;
    out.d_counts = out.mail = nullptr;
    out.pending = false;
    out.n = 0;
    out.counts.assign(B, 0);
    const uint8_t* fr = frames;
    if (!on_dev) {
        uint8_t* d = m.ar.get<uint8_t>(S_FRAMES, (size_t)B * H * W * 3);
        for (int b = 0; b < B; b++)
            VTF_HIP(hipMemcpy2DAsync(d + (size_t)b * H * W * 3, (size_t)W * 3, frames + b * fstride, rstride,
                                     (size_t)W * 3, H, hipMemcpyHostToDevice, st));
        fr = d;
        fstride = (int64_t)H * W * 3;
        rstride = (int64_t)W * 3;
    }
    // ---------------- stage 1: pyramid + PNet (one launch), candidates
    std::vector<PNetLevel> lv;
    int64_t tiles = 0, cells = 0;
    plan_levels(B, H, W, minsize, lv, tiles, cells);
    const int NL = (int)lv.size();
    m.stats[0] = NL;
    m.s1_keys.clear();
    if (NL == 0) return;
    VTF_CHECK(NL < 4096 && cells < (int64_t)1 << 31, VTF_E_LIMIT, "mtcnn: pyramid too large for one call");
    VTF_CHECK(B <= 4096, VTF_E_LIMIT, "mtcnn: at most 4096 frames per call");
    // counters: [0] candidates, [1..NL] per level, [NL+1..NL+3] the PNet launches' tile counters
    // -- zeroed by the SAT row pass (the first launch of the det-batch)
    uint32_t* d_cnt = m.ar.get<uint32_t>(S_COUNT, NL + 4);
    // downsampled levels whose adaptive-pool bins exceed 2 frame pixels are resampled by a
    // separate fully parallel kernel (one thread per level value) into HBM; inside the fused
    // tile kernel their long serial bin sums would leave a few workgroups as a long tail.
    // summed-area table of the preprocessed frames: O(1) exact bin sums for the downsampled
    // levels and the stage-2/3 candidate crops
    // (12 B per entry allocated: either layout fits)
    int3* sat = m.ar.get<int3>(S_SAT, (size_t)B * (H + 1) * (W + 1));
    {
        int min_lh = H, min_lw = W;
        for (auto& L : lv) min_lh = std::min(min_lh, L.lh), min_lw = std::min(min_lw, L.lw);
        m.sat_pk = sat_pack_ok(H, W, min_lh, min_lw) ? 1 : 0;
    }
    launch_sat(fr, fstride, rstride, B, H, W, sat, st, d_cnt, NL + 4, m.sat_pk);
    {
        // split mode: every downsampled level is precomputed as fp16 split pixels (12 B; k_pnet's
        // fill is then a straight 12-byte copy -- the in-kernel bin sums of these levels were
        // latency-bound on 7-14 KB frame patches: 10k + 19k of ~68k workgroup cycles per tile);
        // fp32 mode: only the large-bin levels (H > 2 lh), as fp32 planes
        const bool split = m.pw.c3h != nullptr;
        auto is_pre = [&](const PNetLevel& L) {
            return split ? (L.lh < H || L.lw < W) : (int64_t)H > 2 * (int64_t)L.lh;
        };
        int64_t pre_elems = 0;
        for (auto& L : lv)
            if (is_pre(L)) pre_elems += (int64_t)B * 3 * L.lh * L.lw;  // 12 B per pixel either way
        float* pre = pre_elems ? m.ar.get<float>(S_PRE, pre_elems) : nullptr;
        ResampleLevels rl{};
        rl.split = split ? 1 : 0;
        rl.pk = m.sat_pk;
        for (auto& L : lv) {
            L.pre = nullptr;
            L.pad = 0;
            if (is_pre(L)) {
                L.pad = rl.split;
                VTF_CHECK(rl.n < ResampleLevels::MAXL, VTF_E_LIMIT, "mtcnn: too many precomputed levels");
                L.pre = pre;
                rl.lh[rl.n] = L.lh;
                rl.lw[rl.n] = L.lw;
                rl.out[rl.n] = pre;
                rl.beg[rl.n + 1] = rl.beg[rl.n] + (int64_t)B * L.lh * L.lw;
                rl.n++;
                pre += (int64_t)B * 3 * L.lh * L.lw;
            }
        }
        launch_resample_sat_multi(sat, B, H, W, rl, st);
    }
    // the level plan (and the precomputed levels' addresses in it) is uploaded only when it
    // changes: a video's det-batches share one frame size
    PNetLevel* d_lv = m.ar.get<PNetLevel>(S_LVC, NL);
    if (m.lv_dev != d_lv || m.lv_host.size() != lv.size() ||
        std::memcmp(m.lv_host.data(), lv.data(), lv.size() * sizeof(PNetLevel)) != 0) {
        VTF_HIP(hipMemcpyAsync(d_lv, lv.data(), NL * sizeof(PNetLevel), hipMemcpyHostToDevice, st));
        m.lv_host = lv;
        m.lv_dev = d_lv;
    }
    PNetOut po{};
    po.count = d_cnt;
    po.level_count = d_cnt + 1;
    po.cap = (uint32_t)cells;
    po.key = m.ar.get<uint64_t>(S_KEY, cells);
    po.score = m.ar.get<float>(S_SCORE, cells);
    po.regv = m.ar.get<float4>(S_REGV, cells);
    if (const char* e = getenv("VTF_PNET_DEBUG")) po.dbg = atoi(e);
    // (phase clocks: [0, 8) the exact-levels launch, [8, 16) the general one)
    if (po.dbg & 256) po.clk = m.ar.get<unsigned long long>(S_CLK, 16);
    if (po.clk) VTF_HIP(hipMemsetAsync(po.clk, 0, 128, st));
    const int64_t x_tiles = pnet_exact_tiles(lv, H, W, tiles);
    // one vertical-reuse slot per workgroup of the exact-levels or the PR launch (the same grid
    // rule; the two run one after the other on the stream and share the slots)
    // (allocated only when the opt-in variant is on: VTF_PNET_VR=1, read per det-batch as
    // launch_pnet reads it)
    const char* vre = std::getenv("VTF_PNET_VR");
    const bool vr_on = vre && std::atoi(vre) != 0;
    po.vr_slots = vr_on ? std::max(pnet_x_grid(x_tiles), pnet_x_grid(tiles - pnet_pre_from(lv, tiles))) : 0;
    if (po.vr_slots > 0) po.vr = (uint8_t*)m.ar.get(S_VR, (size_t)po.vr_slots * PNET_VR_SLOT);
    static const bool lowprio = [] {
        const char* e = std::getenv("VTF_PNET_PRIO");
        return e && std::atoi(e) != 0;
    }();
    hipStream_t pst = st;
    if (lowprio) {
        if (!m.pst) {
            int lo = 0, hi = 0;
            VTF_HIP(hipDeviceGetStreamPriorityRange(&lo, &hi));
            VTF_HIP(hipStreamCreateWithPriority(&m.pst, hipStreamNonBlocking, lo));
            VTF_HIP(hipEventCreateWithFlags(&m.pev[0], hipEventDisableTiming));
        }
        pst = m.pst;
        VTF_HIP(hipEventRecord(m.pev[0], st));
        VTF_HIP(hipStreamWaitEvent(pst, m.pev[0], 0));
    }
    if (m.prof) VTF_HIP(hipEventRecord(m.ev0, pst));
    launch_pnet(false, fr, fstride, rstride, H, W, d_lv, NL, tiles, m.pw, po, d_cnt + NL + 1, pst,
                x_tiles, pnet_pre_from(lv, tiles));
    if (m.prof) VTF_HIP(hipEventRecord(m.ev1, pst));
    Arena::Mail mc = m.ar.mail(M_COUNT, (size_t)(NL + 1) * 4);
    k_mail_u32<<<1, 256, 0, pst>>>(d_cnt, (uint32_t*)mc.d, NL + 1);
    VTF_HIP(hipStreamSynchronize(pst));  // (the host sync joins pst back: st's later work follows it)
    std::vector<uint32_t> cnt((const uint32_t*)mc.h, (const uint32_t*)mc.h + NL + 1);
    if (po.clk) {  // debug: average workgroup clocks per tile and phase (k_pnet mark() points)
        unsigned long long c[16];
        d2h_sync(c, po.clk, 128, st);
        static const char* nm[7] = {"tail", "head", "stage", "fill", "conv1", "conv2", "conv3+heads"};
        fprintf(stderr, "k_pnet phase clocks per tile (%lld tiles):", (long long)tiles);
        for (int k = 0; k < 7; k++) fprintf(stderr, " %s %.0f", nm[k], (double)(c[k] + c[8 + k]) / (double)tiles);
        fprintf(stderr, "\n");
        const int64_t xt = std::min(x_tiles, tiles), gt = tiles - xt;
        for (int v = 0; v < 2; v++) {
            const int64_t nt = v ? gt : xt;
            if (nt <= 0) continue;
            fprintf(stderr, "  %s variant (%lld tiles):", v ? "general" : "exact-levels", (long long)nt);
            for (int k = 0; k < 7; k++) fprintf(stderr, " %s %.0f", nm[k], (double)c[8 * v + k] / (double)nt);
            fprintf(stderr, "\n");
        }
    }
    if (m.prof) {
        float ms = 0.f;
        VTF_HIP(hipEventElapsedTime(&ms, m.ev0, m.ev1));
        m.prof_ms += ms;
        m.prof_launches += 1;
        m.prof_frames += B;
        m.prof_flops += pnet_flops(lv) * B;
    }
    const int64_t n1 = cnt[0];
    m.stats[1] = n1;
    if (n1 == 0) return;
    // order candidates by (level, b, h, w) == reference nonzero() order, level by level
    int32_t* slot = m.ar.get<int32_t>(S_SLOT, n1);
    int32_t* slot2 = m.ar.get<int32_t>(S_SLOT2, n1);
    uint64_t* key2 = m.ar.get<uint64_t>(S_KEY2, n1);
    k_iota<<<cdiv(n1, 256), 256, 0, st>>>(slot, n1);
    int lvl_bits = 1;
    while ((1 << lvl_bits) < NL) lvl_bits++;
    sort_u64_pairs(m.ar, S_SORT, po.key, key2, slot, slot2, n1, 32 + lvl_bits, st);
    if (m.keep_s1) {  // (tests only: one extra sync)
        m.s1_keys.resize(n1);
        VTF_HIP(hipMemcpyAsync(m.s1_keys.data(), key2, n1 * 8, hipMemcpyDeviceToHost, st));
        VTF_HIP(hipStreamSynchronize(st));
    }
    float4* b1 = m.ar.get<float4>(S_B1, n1);
    float* s1 = m.ar.get<float>(S_S1, n1);
    float4* r1 = m.ar.get<float4>(S_R1, n1);
    int32_t* i1 = m.ar.get<int32_t>(S_I1, n1);
    int32_t* c1 = m.ar.get<int32_t>(S_C1, n1);
    launch_decode_stage1(key2, slot2, po.score, po.regv, d_lv, n1, b1, s1, r1, i1, c1, st);
    // per-level batched_nms(0.5) (mtcnn.py:196)
    std::vector<int64_t> calls(NL), nk;
    for (int l = 0; l < NL; l++) calls[l] = cnt[l + 1];
    int32_t* keep = m.ar.get<int32_t>(S_KEEP, n1);
    nms_multi(m.ar, (const float*)b1, s1, i1, c1, calls, B, 0.5, keep, nk, st);
    int64_t k1 = std::accumulate(nk.begin(), nk.end(), (int64_t)0);
    m.stats[2] = k1;
    // concatenate levels (keep order) -> batched_nms(0.7) (mtcnn.py:203-206); the gather also
    // zeroes the single call's ids
    float4* b2 = m.ar.get<float4>(S_B2, k1);
    float* s2 = m.ar.get<float>(S_S2, k1);
    float4* r2 = m.ar.get<float4>(S_R2, k1);
    int32_t* i2 = m.ar.get<int32_t>(S_I2, k1);
    int32_t* c2 = m.ar.get<int32_t>(S_C2, k1);
    launch_gather_refine(keep, k1, b1, s1, r1, i1, 0, 0, 0, b2, s2, r2, i2, st, c2);
    nms_multi(m.ar, (const float*)b2, s2, i2, c2, {k1}, B, 0.7, keep, nk, st);
    int64_t k2 = nk[0];
    m.stats[3] = k2;
    if (k2 == 0) return;
    // refine(plus_one=False) + square (mtcnn.py:207-208) -> stage-2 proposals; the launch zeroes
    // the stage's guard and error words
    int32_t* err = m.d_ovf + 2;
    launch_gather_refine(keep, k2, b2, s2, r2, i2, 1, 0, 1, b1, s1, nullptr, i1, st, nullptr, m.d_ovf, 4);
    // ---------------- stage 2: crop 24x24 + RNet (mtcnn.py:213-222)
    float* prob = m.ar.get<float>(S_PROB, k2);
    float4* reg = m.ar.get<float4>(S_REG, k2);
    int32_t* idx = m.ar.get<int32_t>(S_IDX, k2);
    int32_t ctl[3];
    bool deferred = false;
    cand_nets(m, false, sat, H, W, b1, i1, k2, reg, nullptr, prob, err, &deferred);
    int64_t n2 = threshold_compact(m, prob, k2, 0.7f, idx, ctl);
    if (deferred && ctl[0]) {  // the guarded split path tripped: RNet again in fp32
        cand_rerun_fp32(m, false, sat, H, W, b1, i1, k2, reg, nullptr, prob, err);
        n2 = threshold_compact(m, prob, k2, 0.7f, idx, ctl);
    }
    VTF_CHECK(ctl[2] == 0, VTF_E_DEGENERATE,
              "stage 2: a candidate box lies outside the frame; the reference skips it in "
              "_get_cropped_candidates (mtcnn.py:159) and then fails indexing (IndexError)");
    m.stats[4] = n2;
    if (n2 == 0) return;
    launch_gather_refine(idx, n2, b1, prob, reg, i1, 0, 0, 0, b2, s2, r2, i2, st, c2);
    nms_multi(m.ar, (const float*)b2, s2, i2, c2, {n2}, B, 0.7, keep, nk, st);
    int64_t k3 = nk[0];
    m.stats[5] = k3;
    if (k3 == 0) return;
    launch_gather_refine(keep, k3, b2, s2, r2, i2, 1, 1, 1, b1, s1, nullptr, i1, st, nullptr, m.d_ovf, 4);
    // ---------------- stage 3: crop 48x48 + ONet (mtcnn.py:228-242)
    prob = m.ar.get<float>(S_PROB, k3);
    reg = m.ar.get<float4>(S_REG, k3);
    float* lm = m.ar.get<float>(S_LM, k3 * 10);
    idx = m.ar.get<int32_t>(S_IDX, k3);
    deferred = false;
    cand_nets(m, true, sat, H, W, b1, i1, k3, reg, lm, prob, err, &deferred);
    int64_t n3 = threshold_compact(m, prob, k3, 0.7f, idx, ctl);
    if (deferred && ctl[0]) {  // the guarded split path tripped: ONet again in fp32
        cand_rerun_fp32(m, true, sat, H, W, b1, i1, k3, reg, lm, prob, err);
        n3 = threshold_compact(m, prob, k3, 0.7f, idx, ctl);
    }
    VTF_CHECK(ctl[2] == 0, VTF_E_DEGENERATE,
              "stage 3: a candidate box lies outside the frame; the reference skips it in "
              "_get_cropped_candidates (mtcnn.py:159) and then fails indexing (IndexError)");
    m.stats[6] = n3;
    if (n3 == 0) return;
    launch_gather_refine(idx, n3, b1, prob, reg, i1, 0, 0, 0, b2, s2, r2, i2, st);
    float* lmr = m.ar.get<float>(S_LMK, n3 * 10);
    k_gather_rows<<<cdiv(n3 * 10, 256), 256, 0, st>>>(idx, n3, lm, 10, lmr);
    float* lmk = m.ar.get<float>(S_OUTL, n3 * 10);
    launch_landmarks(b2, lmr, n3, lmk, st);
    // refine(+1) without square, then IoM chain NMS (mtcnn.py:241-242)
    float4* b3 = m.ar.get<float4>(S_B1, n3);
    launch_gather_refine(nullptr, n3, b2, nullptr, r2, nullptr, 1, 1, 0, b3, nullptr, nullptr, nullptr, st);
    uint64_t* kk = m.ar.get<uint64_t>(S_KEY2, n3);
    uint64_t* kk2 = m.ar.get<uint64_t>(S_KEY, n3);
    int32_t* io = m.ar.get<int32_t>(S_SLOT, n3);
    int32_t* order = m.ar.get<int32_t>(S_SLOT2, n3);
    k_desc_keys<<<cdiv(n3, 256), 256, 0, st>>>(s2, n3, kk);
    k_iota<<<cdiv(n3, 256), 256, 0, st>>>(io, n3);
    sort_u64_pairs(m.ar, S_SORT, kk, kk2, io, order, n3, 32, st);
    int32_t* kflag = m.ar.get<int32_t>(S_FLAG, n3);
    launch_iom_chain(b3, i2, order, n3, 0.7f, kflag, st);
    int32_t* incl = m.ar.get<int32_t>(S_INCL, n3);
    inclusive_scan_i32(m.ar, S_SCAN, kflag, incl, n3, st);
    int32_t* pos = m.ar.get<int32_t>(S_IDX, n3);
    launch_flag_compact(kflag, incl, n3, pos, st);
    // final rows grouped by image in IoM keep order (element of keep row k = order[pos[k]]),
    // sized by the n3 bound; the kept count is read on the device (incl[n3 - 1]) and, with the
    // per-image counts, reaches the host through the mailbox at the caller's sync
    float* rows = m.ar.get<float>(S_OUTB, (size_t)n3 * 5);
    float* lmo = m.ar.get<float>(S_OUTS, (size_t)n3 * 10);
    int32_t* dcnt = m.ar.get<int32_t>(S_OUTI, B);
    Arena::Mail mr = m.ar.mail(M_ROWS, (size_t)(B + 1) * 4);
    k_mtcnn_rows<<<1, 1024, 0, st>>>(order, pos, incl + n3 - 1, i2, b3, s2, lmk, B, rows, lmo, dcnt, (int32_t*)mr.d);
    out.rows = rows;
    out.lms = lmo;
    out.d_counts = dcnt;
    out.mail = (const int32_t*)mr.h;
    out.pending = true;
}

}  // namespace vtf

using namespace vtf;

struct vtf_mtcnn_s {
    Mtcnn m;
};

extern "C" {

int vtf_mtcnn_create(const float* params, int64_t n_params, int device, vtf_mtcnn_t* out) {
    return guarded([&] {
        VTF_CHECK(params && out, VTF_E_ARG, "null argument");
        DeviceGuard dg(device);
        auto* h = new vtf_mtcnn_s();
        h->m.device = device;
        try {
            build_weights(h->m, params, n_params);
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
    });
}

int vtf_mtcnn_destroy(vtf_mtcnn_t h) {
    return guarded_on(h ? h->m.device : -1, [&] { delete h; });
}

int vtf_mtcnn_set_stream(vtf_mtcnn_t h, void* stream) {
    return guarded_on(h ? h->m.device : -1, [&] {
        VTF_CHECK(h, VTF_E_ARG, "null handle");
        h->m.st = (hipStream_t)stream;
    });
}

int vtf_mtcnn_stats(vtf_mtcnn_t h, int64_t* out8) {
    return guarded_on(h ? h->m.device : -1, [&] {
        VTF_CHECK(h && out8, VTF_E_ARG, "null argument");
        std::memcpy(out8, h->m.stats, sizeof(h->m.stats));
    });
}

int vtf_mtcnn_stage1_keys(vtf_mtcnn_t h, int enable, uint64_t* out, int64_t cap, int64_t* out_n) {
    return guarded_on(h ? h->m.device : -1, [&] {
        VTF_CHECK(h && out_n && cap >= 0 && (out || cap == 0), VTF_E_ARG, "bad argument");
        Mtcnn& m = h->m;
        if (enable >= 0) m.keep_s1 = enable != 0;
        *out_n = (int64_t)m.s1_keys.size();
        std::memcpy(out, m.s1_keys.data(), (size_t)std::min<int64_t>(cap, *out_n) * 8);
    });
}

int vtf_mtcnn_profile(vtf_mtcnn_t h, int enable, double* out_ms, int64_t* out_launches, double* out_flops,
                      int64_t* out_frames) {
    return guarded_on(h ? h->m.device : -1, [&] {
        VTF_CHECK(h, VTF_E_ARG, "null handle");
        Mtcnn& m = h->m;
        if (out_ms) *out_ms = m.prof_ms;
        if (out_launches) *out_launches = m.prof_launches;
        if (out_flops) *out_flops = m.prof_flops;
        if (out_frames) *out_frames = m.prof_frames;
        if (enable) {
            if (!m.ev0) VTF_HIP(hipEventCreate(&m.ev0));
            if (!m.ev1) VTF_HIP(hipEventCreate(&m.ev1));
            m.prof_ms = m.prof_flops = 0;
            m.prof_launches = m.prof_frames = 0;
        }
        m.prof = enable != 0;
    });
}

int vtf_mtcnn_detect(vtf_mtcnn_t h, const uint8_t* frames, int frames_on_device, int B, int H, int W,
                     int64_t frame_stride, int64_t row_stride, double min_face_size, float* out_boxes,
                     float* out_landmarks, int32_t* out_counts, int64_t cap, int64_t* out_total) {
    return guarded_on(h ? h->m.device : -1, [&] {
        VTF_CHECK(h && frames && out_counts, VTF_E_ARG, "null argument");
        DetectOut r;
        detect(h->m, frames, frames_on_device, B, H, W, frame_stride, row_stride, min_face_size, r);
        if (r.pending) VTF_HIP(hipStreamSynchronize(h->m.st));
        r.settle(h->m);
        if (out_total) *out_total = r.n;
        VTF_CHECK(r.n <= cap, VTF_E_CAPACITY, "output capacity too small");
        std::copy(r.counts.begin(), r.counts.end(), out_counts);
        if (r.n == 0) return;
        if (out_boxes) VTF_HIP(hipMemcpyAsync(out_boxes, r.rows, r.n * 20, hipMemcpyDeviceToHost, h->m.st));
        if (out_landmarks) VTF_HIP(hipMemcpyAsync(out_landmarks, r.lms, r.n * 40, hipMemcpyDeviceToHost, h->m.st));
        VTF_HIP(hipStreamSynchronize(h->m.st));
    });
}

int vtf_mtcnn_detect_crops(vtf_mtcnn_t h, const uint8_t* frames, int frames_on_device, int B, int H, int W,
                           int64_t frame_stride, int64_t row_stride, double min_face_size,
                           const vtf_box_params* params, int32_t frame_offset, int32_t* d_crops,
                           int32_t* out_frame_counts, int64_t cap, int64_t* out_n) {
    return guarded_on(h ? h->m.device : -1, [&] {
        VTF_CHECK(h && frames && params && out_n, VTF_E_ARG, "null argument");
        DetectOut r;
        detect(h->m, frames, frames_on_device, B, H, W, frame_stride, row_stride, min_face_size, r);
        if (!r.pending) {  // no rows: the early exits settle on the host
            rows_to_crops(h->m.ar, S_BOXPOST, r.rows, r.counts, H, W, *params, frame_offset, d_crops, nullptr,
                          out_frame_counts, cap, out_n, h->m.st);
            return;
        }
        // box post-processing straight on the device rows and counts; its per-frame counts and
        // total land in a mailbox, read with the detector's rows in one sync.  Crops past `cap`
        // are counted, not written (the caller retries with the reported size).
        VTF_CHECK(cap <= 0 || d_crops, VTF_E_ARG, "null argument");
        Arena::Mail mb = h->m.ar.mail(M_BOXES, ((size_t)B + 1) * 4);
        int32_t* hb = (int32_t*)mb.h;
        int32_t* db = (int32_t*)mb.d;
        launch_box_post(r.rows, r.d_counts, B, H, W, *params, frame_offset, d_crops, nullptr, db, db + B, h->m.st,
                        std::max<int64_t>(cap, 0));
        VTF_HIP(hipStreamSynchronize(h->m.st));
        r.settle(h->m);
        const int64_t total = hb[B];
        *out_n = total;
        VTF_CHECK(total <= cap, VTF_E_CAPACITY, "crop capacity too small (bound: detector rows)");
        if (out_frame_counts) std::copy(hb, hb + B, out_frame_counts);
    });
}

int vtf_iom_nms(const float* d_boxes, const float* d_scores, const int32_t* d_classes, int64_t n, float thr,
                int64_t* d_keep, int64_t* out_nkeep, void* hip_stream) {
    return guarded_on(stream_device((hipStream_t)hip_stream), [&] {
        VTF_CHECK(out_nkeep && n >= 0 && n < ((int64_t)1 << 31), VTF_E_ARG, "bad argument");
        *out_nkeep = 0;
        if (n == 0) return;
        VTF_CHECK(d_boxes && d_scores && d_classes && d_keep, VTF_E_ARG, "null argument");
        hipStream_t st = (hipStream_t)hip_stream;
        StreamScratch sc = stream_scratch(st);
        Arena& ar = *sc.ar;
        uint64_t* kk = ar.get<uint64_t>(80, n);
        uint64_t* kk2 = ar.get<uint64_t>(81, n);
        int32_t* io = ar.get<int32_t>(82, n);
        int32_t* order = ar.get<int32_t>(83, n);
        int32_t* flag = ar.get<int32_t>(84, n);
        int32_t* incl = ar.get<int32_t>(85, n);
        int32_t* pos = ar.get<int32_t>(86, n);
        k_desc_keys<<<cdiv(n, 256), 256, 0, st>>>(d_scores, n, kk);
        k_iota<<<cdiv(n, 256), 256, 0, st>>>(io, n);
        sort_u64_pairs(ar, 87, kk, kk2, io, order, n, 32, st);
        launch_iom_chain((const float4*)d_boxes, d_classes, order, n, thr, flag, st);
        inclusive_scan_i32(ar, 88, flag, incl, n, st);
        launch_flag_compact(flag, incl, n, pos, st);
        int32_t nf = 0;
        d2h_sync(&nf, incl + n - 1, 4, st);
        k_gather_order<<<cdiv(std::max(nf, 1), 256), 256, 0, st>>>(order, pos, nf, d_keep);
        VTF_HIP(hipStreamSynchronize(st));
        *out_nkeep = nf;
    });
}

int vtf_mtcnn_pnet_level(vtf_mtcnn_t h, const uint8_t* d_frames, int B, int H, int W, int64_t frame_stride,
                         int64_t row_stride, int lh, int lw, float* d_prob, float* d_reg) {
    return guarded_on(h ? h->m.device : -1, [&] {
        VTF_CHECK(h && d_frames && d_prob && d_reg && lh >= 12 && lw >= 12, VTF_E_ARG, "bad argument");
        PNetLevel L{};
        L.lh = lh;
        L.lw = lw;
        L.ph = (lh - 1) / 2 - 4;
        L.pw = (lw - 1) / 2 - 4;
        L.scale = 1.f;
        L.tiles_y = cdiv(L.ph, PNET_TH);
        L.tiles_x = cdiv(L.pw, PNET_TW);
        L.tile_beg = 0;
        L.pre = nullptr;
        VTF_CHECK((int64_t)(L.lh + 1) * H < ((int64_t)1 << 31) && (int64_t)(L.lw + 1) * W < ((int64_t)1 << 31),
                  VTF_E_LIMIT, "mtcnn: pyramid level too large for PNet's 32-bit bin math");
        if ((int64_t)H > 2 * (int64_t)lh) {
            int3* sat = h->m.ar.get<int3>(S_SAT, (size_t)B * (H + 1) * (W + 1));
            const int pk = sat_pack_ok(H, W, lh, lw) ? 1 : 0;
            launch_sat(d_frames, frame_stride, row_stride, B, H, W, sat, h->m.st, nullptr, 0, pk);
            float* pre = h->m.ar.get<float>(S_PRE, (int64_t)B * 3 * lh * lw);
            launch_resample_sat(sat, pk, B, H, W, lh, lw, pre, h->m.st);
            L.pre = pre;
        }
        PNetLevel* d_lv = h->m.ar.get<PNetLevel>(S_LEVELS, 1);
        VTF_HIP(hipMemcpyAsync(d_lv, &L, sizeof(L), hipMemcpyHostToDevice, h->m.st));
        PNetOut po{};
        po.prob = d_prob;
        po.reg = d_reg;
        uint32_t* ctr = h->m.ar.get<uint32_t>(S_COUNT, 4);
        VTF_HIP(hipMemsetAsync(ctr, 0, 12, h->m.st));
        launch_pnet(true, d_frames, frame_stride, row_stride, H, W, d_lv, 1, (int64_t)B * L.tiles_x * L.tiles_y,
                    h->m.pw, po, ctr, h->m.st);
        VTF_HIP(hipStreamSynchronize(h->m.st));
    });
}

int vtf_mtcnn_resample(vtf_mtcnn_t h, const uint8_t* d_frames, int B, int H, int W, int64_t frame_stride,
                       int64_t row_stride, int lh, int lw, float* d_out) {
    return guarded_on(h ? h->m.device : -1, [&] {
        VTF_CHECK(h && d_frames && d_out, VTF_E_ARG, "null argument");
        int3* sat = h->m.ar.get<int3>(S_SAT, (size_t)B * (H + 1) * (W + 1));
        const int pk = sat_pack_ok(H, W, lh, lw) ? 1 : 0;
        launch_sat(d_frames, frame_stride, row_stride, B, H, W, sat, h->m.st, nullptr, 0, pk);
        launch_resample_sat(sat, pk, B, H, W, lh, lw, d_out, h->m.st);
        VTF_HIP(hipStreamSynchronize(h->m.st));
    });
}

int vtf_mtcnn_rnet(vtf_mtcnn_t h, const float* d_in, int64_t n, float* d_reg, float* d_prob) {
    return guarded_on(h ? h->m.device : -1, [&] {
        VTF_CHECK(h && d_in && d_reg && d_prob, VTF_E_ARG, "null argument");
        float* x0 = h->m.ar.get<float>(S_CROP, (size_t)n * 24 * 24 * 8);
        launch_nchw_to_nhwc(d_in, (int)n, 3, 24, 24, 8, x0, false, h->m.st);
        run_candidates(h->m, false, x0, n, (float4*)d_reg, nullptr, d_prob);
        VTF_HIP(hipStreamSynchronize(h->m.st));
    });
}

int vtf_mtcnn_onet(vtf_mtcnn_t h, const float* d_in, int64_t n, float* d_reg, float* d_lm, float* d_prob) {
    return guarded_on(h ? h->m.device : -1, [&] {
        VTF_CHECK(h && d_in && d_reg && d_lm && d_prob, VTF_E_ARG, "null argument");
        float* x0 = h->m.ar.get<float>(S_CROP, (size_t)n * 48 * 48 * 8);
        launch_nchw_to_nhwc(d_in, (int)n, 3, 48, 48, 8, x0, false, h->m.st);
        run_candidates(h->m, true, x0, n, (float4*)d_reg, d_lm, d_prob);
        VTF_HIP(hipStreamSynchronize(h->m.st));
    });
}

}  // extern "C"

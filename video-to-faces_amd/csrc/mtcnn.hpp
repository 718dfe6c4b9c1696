#pragma once
#include <vector>

#include "common.hpp"

namespace vtf {

struct PNetLevel {
    int lh, lw;       // level size (int(H*s+1), int(W*s+1)), mtcnn.py:147
    int ph, pw;       // PNet output size
    float scale;      // fp32(s)
    int tiles_x, tiles_y;
    int pad;          // 1: `pre` holds fp16 split pixels (12 B, k_resample_sat_multi split mode)
    int64_t tile_beg; // first workgroup of this level
    const float* pre; // precomputed level [B][3][lh][lw] (large-bin downsampled levels) or null
};

// All conv weights transposed to [ci][ky][kx][co]; dense weights to [k][out] where noted.
struct PNetW {
    const float *c1w, *c1b, *p1, *c2w, *c2b, *p2, *c3w, *c3b, *p3, *c41w, *c41b, *c42w, *c42b;
    // conv3 as fp16 split planes [2][32][144] (w = w0 + w1 * 2^-11, k = tap * 16 + ci) for the
    // fp16 matrix-core path (copied to LDS per tile); null -> fp32 MFMA path (see k_pnet)
    const uint16_t* c3h;
    const uint16_t* c2h;  // conv2: [2][16][96], the 90 (tap, ci) products packed in 3 k-steps (mtcnn_runtime)
    const uint16_t* c1h;  // conv1: [2][16][64], k = ky * 16 + kx * 4 + c (c = 3, kx = 3, ky = 3, co >= 10 zero)
    // both 1x1 heads as fp16 split planes [2][32 rows][32 k] (rows 0,1 conv4_1, 2..5 conv4_2, the
    // rest zero); k = 16 s + 8 hk + i holds channel 16 s + 8 (i >> 2) + (i & 3) + 4 hk: exactly
    // the conv3 accumulator registers 8 s + i of lane half hk (k_pnet's 32x32x16 conv3), so the
    // heads need no lane movement.  null -> fp32 heads
    const uint16_t* hh;
    // PReLU slope classes (host): bit 0 every conv2 slope in [0, 1], bit 1 every conv3 slope in
    // [0, 1] -- PReLU is then max(v, a v), two instructions instead of three
    int unit_slopes;
    // 1: the exact-levels variant's conv1 on 16x16x32 matrix cores with the main and cross products
    // in one chain (w0 pre-scaled by 2^11 on the device: the host checked 2^11 |w0| < 2^15), 0: the
    // 32x32x16 [w0 | w1] layout (env VTF_PNET_C1K=0)
    int c1k;
};
struct PNetOut {
    // sparse (candidate) mode
    uint32_t* count;
    uint32_t* level_count;
    uint32_t cap;
    uint64_t* key;
    float* score;
    float4* regv;
    // dense (parity) mode
    float* prob;
    float* reg;
    int dbg;  // phase-skip mask for profiling (env VTF_PNET_DEBUG): 1 fill, 2 conv1, 4 conv2, 8 conv3,
              // 16 no candidate output, 32 no heads, 64 no frame-patch staging; 256 = phase clocks
    unsigned long long* clk;  // [8] summed shader clocks per phase over workgroups (null: off)
    // k_pnet's vertical-reuse slots (VR_SLOT = 6144 B per workgroup of the exact-levels or the PR
    // launch) and their count: with env VTF_PNET_VR=1 launch_pnet runs the reuse variants when
    // their grid fits (opt-in: measured neutral)
    uint8_t* vr;
    int64_t vr_slots;
};
constexpr int PNET_VR_SLOT = 6144;

// the det-batch's summed-area table (mtcnn_dev.hpp): int3 entries, or packed uint64 (pk) when
// sat_pack_ok says every bin the det-batch reads is small enough
void launch_sat(const uint8_t* frames, int64_t frame_stride, int64_t row_stride, int B, int H, int W, void* sat,
                hipStream_t st, uint32_t* zero = nullptr, int nzero = 0, int pk = 0);
bool sat_pack_ok(int H, int W, int min_lh, int min_lw);
void launch_resample_sat(const void* sat, int pk, int B, int H, int W, int lh, int lw, float* out, hipStream_t st);
struct ResampleLevels {  // precomputed pyramid levels of one det-batch (k_resample_sat_multi)
    static constexpr int MAXL = 32;
    int n;
    int split;  // 1: [B][lh][lw] fp16 split pixels (x0 RGB | x1 RGB, 12 B), else fp32 [B][3][lh][lw]
    int pk;     // the SAT is in the packed layout
    int lh[MAXL], lw[MAXL];
    int64_t beg[MAXL + 1];  // first output element (b, y, x) of each level in the flattened grid
    int64_t tbeg[MAXL + 1]; // first 2-D tile of each level (k_resample_sat_multi's grid; set by the launcher)
    float* out[MAXL];       // [B][3][lh][lw]
};
void launch_resample_sat_multi(const void* sat, int B, int H, int W, const ResampleLevels& lv, hipStream_t st);
void launch_pnet(bool dense, const uint8_t* frames, int64_t frame_stride, int64_t row_stride, int H, int W,
                 const PNetLevel* d_levels, int n_levels, int64_t total_tiles, const PNetW& w, const PNetOut& o,
                 uint32_t* d_tile_ctr, hipStream_t st, int64_t exact_tiles = 0,
                 int64_t pre_from = INT64_MAX);  // d_tile_ctr: 3 zeroed words
// grid of k_pnet's exact-levels launch over that many tiles (= vertical-reuse slots it needs)
int64_t pnet_x_grid(int64_t exact_tiles);
// first tile of the trailing levels precomputed as fp16 split pixels (k_pnet's PR variant)
int64_t pnet_pre_from(const std::vector<PNetLevel>& lv, int64_t total_tiles);
// leading tiles of the level plan that k_pnet's exact-levels variant takes (see launch_pnet)
int64_t pnet_exact_tiles(const std::vector<PNetLevel>& lv, int H, int W, int64_t total_tiles);
int cand_front_side(bool onet);
void launch_cand_front(bool onet, const void* sat, int pk, int H, int W, const float4* boxes, const int32_t* img,
                       int64_t n, const float* w1, const _Float16* w1h, const float* b1, const float* a1, float* out,
                       int32_t* err, hipStream_t st, int* ovf = nullptr);
// Fused RNet / ONet front half (mtcnn_cand.hip): crop + conv1 + PReLU + pool + conv2 + PReLU +
// pool on split-fp16 matrix cores -> pool2 map [n, P2, P2, 48 | 64] fp32 (P2 = 4 | 10).
// w1h: conv1 split planes [2][32][64] (k = ky*16 + kx*4 + c), w2h: conv2 [2][C2][288]
// (k = (ky*3 + kx)*32 + ci); b/a: bias / PReLU slope padded to 32 / C2.
struct CandFusedW {
    const _Float16* w1h;
    const float *b1, *a1;
    const _Float16* w2h;
    const float *b2, *a2;
};
int cand_fused_side(bool onet);
void launch_cand_fused(bool onet, const void* sat, int pk, int H, int W, const float4* boxes, const int32_t* img,
                       int64_t n, const CandFusedW& w, float* out, int32_t* err, int32_t* ovf, hipStream_t st);
void launch_heads(const float* x, int64_t n, int D, const float* w1, const float* b1, const float* w2,
                  const float* b2, const float* w3, const float* b3, float* prob, float4* reg, float* lm,
                  hipStream_t st);
void launch_decode_stage1(const uint64_t* key_sorted, const int32_t* slot_sorted, const float* score,
                          const float4* regv, const PNetLevel* lv, int64_t n, float4* boxes, float* sc, float4* reg,
                          int32_t* img, int32_t* call, hipStream_t st);
void launch_gather_refine(const int32_t* idx, int64_t n, const float4* bin, const float* sin, const float4* rin,
                          const int32_t* iin, int refine, int plus_one, int square, float4* bout, float* sout,
                          float4* rout, int32_t* iout, hipStream_t st, int32_t* zout = nullptr,
                          int32_t* zw = nullptr, int nzw = 0);
void launch_threshold(const float* s, int64_t n, float thr, int32_t* flag, hipStream_t st);
void launch_flag_compact(const int32_t* flag, const int32_t* incl, int64_t n, int32_t* out, hipStream_t st,
                         int32_t* mail = nullptr, const int32_t* ctl = nullptr, int nctl = 0);
void launch_landmarks(const float4* boxes, const float* lm, int64_t n, float* out, hipStream_t st);
void launch_iom_chain(const float4* boxes, const int32_t* img, const int32_t* order, int64_t n, float thr,
                      int32_t* keep, hipStream_t st);

constexpr int PNET_TH = 16, PNET_TW = 16;  // k_pnet output cells per tile (rows, cols)

}  // namespace vtf

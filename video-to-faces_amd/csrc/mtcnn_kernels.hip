// MTCNN kernels for gfx950 (fp32-grade; parity with the reference PyTorch-CPU path).
//
// Reference: src/videotofaces/detectors/mtcnn.py
//   _preprocess 133-139, _resample 150-151, PNet 12-38, stage-1 candidates 183-194,
//   _get_cropped_candidates 153-163, RNet 41-76, ONet 79-121.
//
// MI355X design:
//   * k_pnet: ONE persistent launch per det-batch covers every pyramid level of every frame.
//     Each 256-thread workgroup (3 per CU) takes PNET_TH x PNET_TW (16x16) tiles of PNet output
//     cells from a chunked atomic counter.  The level pixels a tile needs ((2TH+10)^2 x 3) are
//     computed on the fly from the uint8 BGR frame (preprocess + adaptive_avg_pool2d,
//     bit-exact: the bin sums are exact integers) straight into LDS, so the 10.7 Mpx/frame
//     pyramid never exists in HBM (large-bin downsampled levels come from the frame's
//     summed-area table, k_resample_sat).  conv1 + PReLU + maxpool(ceil), conv2 + PReLU,
//     conv3 + PReLU and both 1x1 heads run on the fp16 matrix cores with split operands
//     (x = x0 + x1 * 2^-11, fp32-grade products), with fp32 MFMA / VALU fallbacks
//     when the host cannot bound the activations to the fp16 range.  Cells with p >= 0.6 are
//     appended with one wave-aggregated atomic -- the dense prob/reg maps are never written.
//   * k_cand_front: one workgroup per candidate box; the crop + adaptive pool to 24x24 / 48x48
//     from the SAT (replacing the reference's per-box Python loop) feeds conv1 + PReLU + the
//     ceil max-pool in LDS; the rest of RNet / ONet runs on the conv kernel (conv.hip).
// Build with -ffp-contract=off: only explicit fmaf() fuses.
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "common.hpp"
#include "mtcnn.hpp"
#include "mtcnn_dev.hpp"

namespace vtf {

typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;

// ----------------------------------------------------------------------------------- helpers

// Summed-area table of the preprocessed frame.  (u - 127.5) / 128 = (2u - 255) / 256 is exact
// in fp32, and so is every partial sum of such values over an adaptive-pool bin (|sum| < 2^16
// with 8 fractional bits), so the reference's sequential fp32 bin sum (adaptive_avg_pool2d,
// row-major) equals the integer box sum of v = 2u - 255 times 2^-8, bit for bit.
// sat[b][y][x] = (R, G, B) sums over rows < y, cols < x; y in [0,H], x in [0,W], as 12-byte int3
// or, when every bin of the det-batch is small enough, 8-byte packed entries (mtcnn_dev.hpp): the
// SAT passes and every corner read are HBM / MALL-bound.

// bin average from an exact integer bin sum: s / kh / kw with the reference's roundings
// PNet weight layout (mtcnn_runtime.hip build_weights checks it): the fp32 tensors are packed
// from PNetW::c1w in state_dict order, each padded to 4 floats; the fp16 split planes from
// PNetW::c3h (conv3, conv2, conv1, heads).  k_pnet addresses everything from the two bases
// with constant offsets: 2 pointers instead of 17 live across the persistent loop (the kernel
// was spilling SGPRs into VGPR lanes).
constexpr int PW_C1W = 0, PW_C1B = 272, PW_P1 = 284, PW_C2W = 296, PW_C2B = 1736, PW_P2 = 1752, PW_C3W = 1768,
              PW_C3B = 6376, PW_P3 = 6408, PW_C41W = 6440, PW_C41B = 6504, PW_C42W = 6508, PW_C42B = 6636,
              PW_F32 = 6640;
constexpr int PH_C2H = 9216, PH_C1H = 12288, PH_HH = 14336;  // halves (conv3 planes at 0)

// ----------------------------------------------------------------------------------- resample

// fp16 split of an fp32 value: v = x0 + x1 * 2^-11 to ~2^-24 relative (x0 = fp16(v), the
// residual v - x0 exact in fp32), the operand form of k_pnet's fp16 matrix-core convolutions
__device__ inline void split_f16(float v, _Float16& x0, _Float16& x1) {
    x0 = (_Float16)v;
    x1 = (_Float16)((v - (float)x0) * 2048.f);
}

// row pass: block per frame row
__global__ __launch_bounds__(256) void k_sat_rows(const uint8_t* __restrict__ frames, int64_t frame_stride,
                                                  int64_t row_stride, int H, int W, int3* __restrict__ sat,
                                                  uint32_t* __restrict__ zero, int nzero) {
    // (folded memset: the det-batch's PNet candidate counters)
    if (blockIdx.x == 0)
        for (int i = threadIdx.x; i < nzero; i += 256) zero[i] = 0u;
    // row prefix sums in passes of 256 consecutive pixels (one per thread: coalesced byte loads
    // and 3 KB contiguous 12-byte stores), a block scan per pass with the carry in registers
    const int y = blockIdx.x % H, b = blockIdx.x / H;
    const int W1 = W + 1;
    const uint8_t* row = frames + (int64_t)b * frame_stride + (int64_t)y * row_stride;
    int3* out = sat + ((int64_t)b * (H + 1) + y + 1) * W1;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ int3 wt[2][4];
    int3 carry = make_int3(0, 0, 0);
    // bytes of the next pass loaded before the current one is scanned
    int nr = 0, ng = 0, nb = 0;
    if (tid < W) {
        nr = 2 * row[3 * tid + 2] - 255;
        ng = 2 * row[3 * tid + 1] - 255;
        nb = 2 * row[3 * tid] - 255;
    }
    for (int x0 = 0, it = 0; x0 < W; x0 += 256, it++) {
        int r = nr, g = ng, bl = nb;
        const int xn = x0 + 256 + tid;
        nr = ng = nb = 0;
        if (xn < W) {
            nr = 2 * row[3 * xn + 2] - 255;
            ng = 2 * row[3 * xn + 1] - 255;
            nb = 2 * row[3 * xn] - 255;
        }
        for (int off = 1; off < 64; off <<= 1) {  // inclusive wave scan
            const int tr = __shfl_up(r, off), tg = __shfl_up(g, off), tb = __shfl_up(bl, off);
            if (lane >= off) {
                r += tr;
                g += tg;
                bl += tb;
            }
        }
        if (lane == 63) wt[it & 1][wave] = make_int3(r, g, bl);  // double-buffered: one barrier per pass
        __syncthreads();
        int3 wb = carry;
        for (int w = 0; w < 4; w++) {
            const int3 t = wt[it & 1][w];
            if (w < wave) {
                wb.x += t.x;
                wb.y += t.y;
                wb.z += t.z;
            }
            carry.x += t.x;
            carry.y += t.y;
            carry.z += t.z;
        }
        const int x = x0 + tid;
        if (x < W) out[x + 1] = make_int3(wb.x + r, wb.y + g, wb.z + bl);
    }
    if (tid == 0) out[0] = make_int3(0, 0, 0);
    if (y == 0) {
        int3* r0 = sat + (int64_t)b * (H + 1) * W1;
        for (int x = tid; x < W1; x += 256) r0[x] = make_int3(0, 0, 0);
    }
}

// column pass, in place: block = 16 columns x G row groups of up to SAT_PER rows; each thread
// keeps its rows in registers (the SAT is read once and written once), group totals combined
// in LDS
constexpr int SAT_COLS = 16, SAT_PER = 24, SAT_MAXG = 64;
__global__ __launch_bounds__(SAT_COLS * SAT_MAXG) void k_sat_cols(int H, int W, int3* __restrict__ sat) {
    const int W1 = W + 1;
    const int G = blockDim.x / SAT_COLS;
    const int ncb = (W1 + SAT_COLS - 1) / SAT_COLS;
    const int b = blockIdx.x / ncb, cb = blockIdx.x % ncb;
    const int c = threadIdx.x % SAT_COLS, g = threadIdx.x / SAT_COLS;
    const int x = cb * SAT_COLS + c;
    const int per = (H + G - 1) / G;
    const int ys = 1 + g * per, ye = min(H + 1, ys + per);
    int3* col = sat + (int64_t)b * (H + 1) * W1 + min(x, W1 - 1);
    // [G][SAT_COLS] group totals, sized by the launch (7.7 KB at 720p): small enough to co-reside
    // with another lane's persistent k_pnet (3 x 49 KB of the CU's 160 KB), so a det-batch's SAT
    // does not wait for the other lanes' pyramid kernels to drain
    extern __shared__ int3 tot_s[];
    int3 (*tot)[SAT_COLS] = (int3 (*)[SAT_COLS])tot_s;
    int3 v[SAT_PER];
    int3 acc = make_int3(0, 0, 0);
#pragma unroll
    for (int i = 0; i < SAT_PER; i++) {
        v[i] = (x < W1 && ys + i < ye) ? col[(int64_t)(ys + i) * W1] : make_int3(0, 0, 0);
        acc.x += v[i].x;
        acc.y += v[i].y;
        acc.z += v[i].z;
    }
    tot[g][c] = acc;
    __syncthreads();
    int3 off = make_int3(0, 0, 0);
    for (int k = 0; k < g; k++) {
        off.x += tot[k][c].x;
        off.y += tot[k][c].y;
        off.z += tot[k][c].z;
    }
#pragma unroll
    for (int i = 0; i < SAT_PER; i++) {
        off.x += v[i].x;
        off.y += v[i].y;
        off.z += v[i].z;
        if (x < W1 && ys + i < ye) col[(int64_t)(ys + i) * W1] = off;
    }
}

// the packed layout (mtcnn_dev.hpp): the same two passes on uint64 prefix sums of packed u
// (8 B per entry instead of 12: the passes and every corner read move two thirds of the bytes)
__global__ __launch_bounds__(256) void k_sat_rows_pk(const uint8_t* __restrict__ frames, int64_t frame_stride,
                                                     int64_t row_stride, int H, int W, uint64_t* __restrict__ sat,
                                                     uint32_t* __restrict__ zero, int nzero) {
    if (blockIdx.x == 0)
        for (int i = threadIdx.x; i < nzero; i += 256) zero[i] = 0u;
    const int y = blockIdx.x % H, b = blockIdx.x / H;
    const int W1 = W + 1;
    const uint8_t* row = frames + (int64_t)b * frame_stride + (int64_t)y * row_stride;
    uint64_t* out = sat + ((int64_t)b * (H + 1) + y + 1) * W1;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    __shared__ uint64_t wt[2][4];
    uint64_t carry = 0, np = tid < W ? sat_pack_px(row + 3 * tid) : 0;
    for (int x0 = 0, it = 0; x0 < W; x0 += 256, it++) {
        uint64_t p = np;
        const int xn = x0 + 256 + tid;
        np = xn < W ? sat_pack_px(row + 3 * xn) : 0;
        for (int off = 1; off < 64; off <<= 1) {  // inclusive wave scan
            const uint64_t t = __shfl_up(p, off);
            if (lane >= off) p += t;
        }
        if (lane == 63) wt[it & 1][wave] = p;
        __syncthreads();
        uint64_t wb = carry;
        for (int w = 0; w < 4; w++) {
            const uint64_t t = wt[it & 1][w];
            if (w < wave) wb += t;
            carry += t;
        }
        const int x = x0 + tid;
        if (x < W) out[x + 1] = wb + p;
    }
    if (tid == 0) out[0] = 0;
    if (y == 0) {
        uint64_t* r0 = sat + (int64_t)b * (H + 1) * W1;
        for (int x = tid; x < W1; x += 256) r0[x] = 0;
    }
}

// one WAVE per frame row (4 rows per workgroup, no workgroup barrier), staged through the wave's
// LDS slice both ways so every global access is lane-contiguous: the row's bytes in as dwords, the
// lane's 20 consecutive pixels packed and prefix-summed in registers, one wave scan of the lane
// totals, the row's 1281 sums out as 8-byte stores.  For W <= 1280 with 4-byte aligned rows and
// W * 3 % 4 == 0 (launch_sat checks).
__device__ inline void wave_lds_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
__global__ __launch_bounds__(256) void k_sat_rows_pkw(const uint8_t* __restrict__ frames, int64_t frame_stride,
                                                      int64_t row_stride, int H, int W, int64_t rows,
                                                      uint64_t* __restrict__ sat, uint32_t* __restrict__ zero,
                                                      int nzero) {
    constexpr int PPL = 20;
    __shared__ uint64_t stage_s[4][64 * PPL];
    if (blockIdx.x == 0)
        for (int i = threadIdx.x; i < nzero; i += 256) zero[i] = 0u;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
    const int64_t rid = (int64_t)blockIdx.x * 4 + wv;
    if (rid >= rows) return;  // (wave-uniform)
    const int y = (int)(rid % H), b = (int)(rid / H);
    const int W1 = W + 1;
    const uint32_t* row = (const uint32_t*)(frames + (int64_t)b * frame_stride + (int64_t)y * row_stride);
    uint64_t* out = sat + ((int64_t)b * (H + 1) + y + 1) * W1;
    uint64_t* stage = stage_s[wv];
    uint32_t* bytes = (uint32_t*)stage;  // the row's bytes first, then the sums
    const int nd = W * 3 / 4;
    for (int d = lane; d < nd; d += 64) bytes[d] = row[d];
    wave_lds_sync();
    const int x0 = lane * PPL;
    uint32_t w[PPL * 3 / 4];
#pragma unroll
    for (int d = 0; d < PPL * 3 / 4; d++) w[d] = x0 * 3 / 4 + d < nd ? bytes[x0 * 3 / 4 + d] : 0u;
    const uint8_t* px = (const uint8_t*)w;
    uint64_t v[PPL], run = 0;
#pragma unroll
    for (int k = 0; k < PPL; k++) {
        run += x0 + k < W ? sat_pack_px(px + 3 * k) : 0;
        v[k] = run;
    }
    uint64_t incl = run;
    for (int off = 1; off < 64; off <<= 1) {
        const uint64_t t = __shfl_up(incl, off);
        if (lane >= off) incl += t;
    }
    const uint64_t excl = incl - run;
    wave_lds_sync();  // every lane has its bytes in registers
#pragma unroll
    for (int k = 0; k < PPL; k++) stage[x0 + k] = excl + v[k];
    wave_lds_sync();
    for (int x = lane; x < W; x += 64) out[x + 1] = stage[x];
    if (lane == 0) out[0] = 0;
    if (y == 0) {
        uint64_t* r0 = sat + (int64_t)b * (H + 1) * W1;
        for (int x = lane; x < W1; x += 64) r0[x] = 0;
    }
}

__global__ __launch_bounds__(SAT_COLS * SAT_MAXG) void k_sat_cols_pk(int H, int W, uint64_t* __restrict__ sat) {
    const int W1 = W + 1;
    const int G = blockDim.x / SAT_COLS;
    const int ncb = (W1 + SAT_COLS - 1) / SAT_COLS;
    const int b = blockIdx.x / ncb, cb = blockIdx.x % ncb;
    const int c = threadIdx.x % SAT_COLS, g = threadIdx.x / SAT_COLS;
    const int x = cb * SAT_COLS + c;
    const int per = (H + G - 1) / G;
    const int ys = 1 + g * per, ye = min(H + 1, ys + per);
    uint64_t* col = sat + (int64_t)b * (H + 1) * W1 + min(x, W1 - 1);
    extern __shared__ uint64_t tot_q[];
    uint64_t (*tot)[SAT_COLS] = (uint64_t (*)[SAT_COLS])tot_q;
    uint64_t v[SAT_PER];
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < SAT_PER; i++) {
        v[i] = (x < W1 && ys + i < ye) ? col[(int64_t)(ys + i) * W1] : 0;
        acc += v[i];
    }
    tot[g][c] = acc;
    __syncthreads();
    uint64_t off = 0;
    for (int k = 0; k < g; k++) off += tot[k][c];
#pragma unroll
    for (int i = 0; i < SAT_PER; i++) {
        off += v[i];
        if (x < W1 && ys + i < ye) col[(int64_t)(ys + i) * W1] = off;
    }
}

// column pass of the packed table for frames up to 1024 rows: 32 columns (256 B per row) x up
// to 32 groups of 32 rows (63.8 -> 52.9 us per 720p det-batch against 16 columns)
constexpr int SATP_COLS = 32, SATP_PER = 32, SATP_MAXG = 32;
__global__ __launch_bounds__(SATP_COLS * SATP_MAXG) void k_sat_cols_pk32(int H, int W, uint64_t* __restrict__ sat) {
    const int W1 = W + 1;
    const int G = blockDim.x / SATP_COLS;
    const int ncb = (W1 + SATP_COLS - 1) / SATP_COLS;
    const int b = blockIdx.x / ncb, cb = blockIdx.x % ncb;
    const int c = threadIdx.x % SATP_COLS, g = threadIdx.x / SATP_COLS;
    const int x = cb * SATP_COLS + c;
    const int per = (H + G - 1) / G;
    const int ys = 1 + g * per, ye = min(H + 1, ys + per);
    uint64_t* col = sat + (int64_t)b * (H + 1) * W1 + min(x, W1 - 1);
    extern __shared__ uint64_t tot_q[];
    uint64_t (*tot)[SATP_COLS] = (uint64_t (*)[SATP_COLS])tot_q;
    uint64_t v[SATP_PER];
    uint64_t acc = 0;
#pragma unroll
    for (int i = 0; i < SATP_PER; i++) {
        v[i] = (x < W1 && ys + i < ye) ? col[(int64_t)(ys + i) * W1] : 0;
        acc += v[i];
    }
    tot[g][c] = acc;
    __syncthreads();
    uint64_t off = 0;
    for (int k = 0; k < g; k++) off += tot[k][c];
#pragma unroll
    for (int i = 0; i < SATP_PER; i++) {
        off += v[i];
        if (x < W1 && ys + i < ye) col[(int64_t)(ys + i) * W1] = off;
    }
}

void launch_sat(const uint8_t* frames, int64_t frame_stride, int64_t row_stride, int B, int H, int W, void* sat,
                hipStream_t st, uint32_t* zero, int nzero, int pk) {
    const int G = (H + SAT_PER - 1) / SAT_PER;
    VTF_CHECK(G <= SAT_MAXG, VTF_E_LIMIT, "mtcnn: frames taller than 1536 rows");
    const unsigned gc = (unsigned)(B * ((W + SAT_COLS) / SAT_COLS));
    if (pk) {
        // (the wave-per-row pass without the LDS staging measured 54.5 -> 79.3 us: per-lane 160-byte
        //  store runs do not coalesce)
        const int64_t rows = (int64_t)B * H;
        if (W <= 1280 && W * 3 % 4 == 0 && frame_stride % 4 == 0 && row_stride % 4 == 0 && ((uintptr_t)frames & 3) == 0)
            k_sat_rows_pkw<<<(unsigned)((rows + 3) / 4), 256, 0, st>>>(frames, frame_stride, row_stride, H, W, rows,
                                                                        (uint64_t*)sat, zero, nzero);
        else
            k_sat_rows_pk<<<(unsigned)rows, 256, 0, st>>>(frames, frame_stride, row_stride, H, W, (uint64_t*)sat, zero,
                                                          nzero);
        const int GP = (H + SATP_PER - 1) / SATP_PER;
        if (GP <= SATP_MAXG)
            k_sat_cols_pk32<<<(unsigned)(B * ((W + SATP_COLS) / SATP_COLS)), SATP_COLS * GP,
                              (size_t)GP * SATP_COLS * sizeof(uint64_t), st>>>(H, W, (uint64_t*)sat);
        else
            k_sat_cols_pk<<<gc, SAT_COLS * G, (size_t)G * SAT_COLS * sizeof(uint64_t), st>>>(H, W, (uint64_t*)sat);
        return;
    }
    k_sat_rows<<<(unsigned)((int64_t)B * H), 256, 0, st>>>(frames, frame_stride, row_stride, H, W, (int3*)sat, zero, nzero);
    k_sat_cols<<<gc, SAT_COLS * G, (size_t)G * SAT_COLS * sizeof(int3), st>>>(H, W, (int3*)sat);
}

// the packed layout is exact for boxes of at most 8223 pixels (255 * area < 2^21 per channel):
// the largest bin a det-batch reads -- the downsampled pyramid levels' bins and the 24 / 48 crops
// of candidate boxes clipped to the frame -- must stay below that (VTF_SAT_PACK=0: int3 always)
bool sat_pack_ok(int H, int W, int min_lh, int min_lw) {
    const char* e = std::getenv("VTF_SAT_PACK");  // (read per det-batch: the tests run both layouts)
    const bool on = !(e && std::atoi(e) == 0);
    auto bin = [](int64_t L, int64_t l) { return (L + l - 1) / l + 1; };
    const int64_t crop = bin(H, 24) * bin(W, 24);
    const int64_t lvl = bin(H, std::max(1, min_lh)) * bin(W, std::max(1, min_lw));
    return on && std::max(crop, lvl) * 255 < ((int64_t)1 << 21);
}

// MTCNN._resample of the preprocessed frames (mtcnn.py:133-139, 150-151) from the SAT:
// out [B][3][lh][lw], one thread per level pixel (all three channels)
__global__ void k_resample_sat(const void* __restrict__ sat, int pk, int B, int H, int W, int lh, int lw,
                               float* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t n = (int64_t)B * lh * lw;
    if (i >= n) return;
    const int lx = (int)(i % lw);
    const int ly = (int)((i / lw) % lh);
    const int b = (int)(i / ((int64_t)lw * lh));
    const int y0 = (int)(((int64_t)ly * H) / lh), y1 = (int)(((int64_t)(ly + 1) * H + lh - 1) / lh);
    const int x0 = (int)(((int64_t)lx * W) / lw), x1 = (int)(((int64_t)(lx + 1) * W + lw - 1) / lw);
    const int3 s = sat_box_any(sat, pk, (int64_t)b * (H + 1) * (W + 1), W + 1, y0, y1, x0, x1);
    const int64_t plane = (int64_t)lh * lw, o = (int64_t)b * 3 * plane + (int64_t)ly * lw + lx;
    out[o] = bin_avg(s.x, y1 - y0, x1 - x0);
    out[o + plane] = bin_avg(s.y, y1 - y0, x1 - x0);
    out[o + 2 * plane] = bin_avg(s.z, y1 - y0, x1 - x0);
}

void launch_resample_sat(const void* sat, int pk, int B, int H, int W, int lh, int lw, float* out, hipStream_t st) {
    int64_t n = (int64_t)B * lh * lw;
    k_resample_sat<<<cdiv(n, 256), 256, 0, st>>>(sat, pk, B, H, W, lh, lw, out);
}

// every precomputed level of a det-batch in one launch (the small levels alone are launch-bound).
// A workgroup takes a 2-D tile of RS_TH level rows x RS_TW pixels (each thread RS_TH / 4 pixels,
// rows r, r + 4, ...): the SAT rows a level row's bins end on are the next row's bin starts, and
// corner columns repeat between neighbours, so a tile's corner reads come from the workgroup's own
// L1 / its XCD's L2 instead of HBM (a row-major strip of 256 pixels per workgroup put the next
// level row on another XCD: 960 MB fetched per det-batch for 260 MB of output)
constexpr int RS_TW = 64;
template <int RS_TH>
__global__ __launch_bounds__(256) void k_resample_sat_multi(const void* __restrict__ sat, int B, int H, int W,
                                                            ResampleLevels lv) {
    const int64_t bid = blockIdx.x;
    int l = 0;
    while (l + 1 < lv.n && bid >= lv.tbeg[l + 1]) l++;
    const int lh = lv.lh[l], lw = lv.lw[l];
    const int txn = (lw + RS_TW - 1) / RS_TW, tyn = (lh + RS_TH - 1) / RS_TH;
    const int64_t t = bid - lv.tbeg[l];
    const int b = (int)(t / ((int64_t)txn * tyn));
    const int tt = (int)(t - (int64_t)b * txn * tyn);
    const int ty = tt / txn, tx = tt - ty * txn;
    const int lx = tx * RS_TW + (threadIdx.x & (RS_TW - 1));
    const int x0 = (int)(((int64_t)lx * W) / lw), x1 = (int)(((int64_t)(lx + 1) * W + lw - 1) / lw);
    const int64_t sb = (int64_t)b * (H + 1) * (W + 1);
#pragma unroll
    for (int h = 0; h < RS_TH / 4; h++) {
        const int ly = ty * RS_TH + (threadIdx.x >> 6) + 4 * h;
        if (ly >= lh || lx >= lw) continue;
        const int64_t j = ((int64_t)b * lh + ly) * lw + lx;
        const int y0 = (int)(((int64_t)ly * H) / lh), y1 = (int)(((int64_t)(ly + 1) * H + lh - 1) / lh);
        const int3 s = sat_box_any(sat, lv.pk, sb, W + 1, y0, y1, x0, x1);
        if (lv.split) {  // fp16 split pixels [B][lh][lw] x (x0 RGB | x1 RGB), k_pnet's level-tile halves
            _Float16 r0, r1, g0, g1, b0, b1;
            split_f16(bin_avg(s.x, y1 - y0, x1 - x0), r0, r1);
            split_f16(bin_avg(s.y, y1 - y0, x1 - x0), g0, g1);
            split_f16(bin_avg(s.z, y1 - y0, x1 - x0), b0, b1);
            // 12 bytes (no pad halves): r0 g0 | b0 r1 | g1 b1
            auto hb = [](_Float16 q) { return (uint32_t)__builtin_bit_cast(uint16_t, q); };
            ((uint3*)lv.out[l])[j] = make_uint3(hb(r0) | hb(g0) << 16, hb(b0) | hb(r1) << 16, hb(g1) | hb(b1) << 16);
            continue;
        }
        const int64_t plane = (int64_t)lh * lw, o = (int64_t)b * 3 * plane + (int64_t)ly * lw + lx;
        float* out = lv.out[l];
        out[o] = bin_avg(s.x, y1 - y0, x1 - x0);
        out[o + plane] = bin_avg(s.y, y1 - y0, x1 - x0);
        out[o + 2 * plane] = bin_avg(s.z, y1 - y0, x1 - x0);
    }
}

void launch_resample_sat_multi(const void* sat, int B, int H, int W, const ResampleLevels& lv0, hipStream_t st) {
    VTF_CHECK(lv0.n >= 0 && lv0.n <= ResampleLevels::MAXL, VTF_E_LIMIT, "mtcnn: too many precomputed levels");
    if (lv0.n == 0 || lv0.beg[lv0.n] == 0) return;
    ResampleLevels lv = lv0;
    // level rows per workgroup tile (VTF_RS_TH = 8 / 16 / 32, read per launch): 32 by default since
    // round 6 -- one SAT row re-read per 32 level rows instead of 8: 655 -> 632 MB fetched, 157 -> 150
    // us per c2 det-batch (profiles/r06_resample_tile_rows_ab.txt)
    const char* e = std::getenv("VTF_RS_TH");
    const int th = e && (std::atoi(e) == 8 || std::atoi(e) == 16) ? std::atoi(e) : 32;
    lv.tbeg[0] = 0;
    for (int l = 0; l < lv.n; l++)
        lv.tbeg[l + 1] = lv.tbeg[l] + (int64_t)B * ((lv.lh[l] + th - 1) / th) * ((lv.lw[l] + RS_TW - 1) / RS_TW);
    VTF_CHECK(lv.tbeg[lv.n] < (int64_t)1 << 31, VTF_E_LIMIT, "mtcnn: resample grid too large");
    if (th == 32) k_resample_sat_multi<32><<<(unsigned)lv.tbeg[lv.n], 256, 0, st>>>(sat, B, H, W, lv);
    else if (th == 16) k_resample_sat_multi<16><<<(unsigned)lv.tbeg[lv.n], 256, 0, st>>>(sat, B, H, W, lv);
    else k_resample_sat_multi<8><<<(unsigned)lv.tbeg[lv.n], 256, 0, st>>>(sat, B, H, W, lv);
}

// ----------------------------------------------------------------------------------- PNet

constexpr int PT_H = PNET_TH, PT_W = PNET_TW;         // output cells per tile (mtcnn.hpp)
static_assert(PT_W % 16 == 0 && (PT_H * PT_W) % 64 == 0, "conv3 fragments are 16-cell row runs, 4 waves");
constexpr int PL_H = 2 * PT_H + 10, PL_W = 2 * PT_W + 10;  // level tile 42 x 42
constexpr int PP_H = PT_H + 4, PP_W = PT_W + 4;       // pooled 20 x 20
constexpr int PC_H = PT_H + 2, PC_W = PT_W + 2;       // conv2 out 18 x 18
constexpr int P_LVL = 3 * PL_H * PL_W;                // 5292
constexpr int P_C2 = 16 * PC_H * PC_W;                // 5184
// pooled conv1: fp32 [10][cells], or fp16 split planes [2][cells][12] (ch 10, 11 zero; conv2 reads
// 8 halves from channel 8 into the next cell, against zero weights) + 4 halves of end padding
constexpr int PQ_C = 12;
constexpr int P_POOL0 = (10 * PP_H * PP_W > PQ_C * PP_H * PP_W) ? 10 * PP_H * PP_W : PQ_C * PP_H * PP_W;
// during conv3 the pooled buffer holds the next tile's first 2 KB of frame patch (floats 0..511)
// and conv3's split weights [2][32][144] halves (floats 512..5119, rows of 72 dwords: conflict-free
// for the 16-byte A-operand reads), so conv3 issues no global loads
constexpr int P_W3 = 512, W3_ROW = 144;
// Bank swizzles for conv3's 16-byte operand reads (ds_read_b128 serves 16 lanes per LDS cycle:
// {0-3,12-15,20-27}, {4-11,16-19,28-31} and the same for lanes 32-63).  C3_SWZ: weight rows
// >= 16 of each plane hold every tap's channel halves swapped ([8..15 | 0..7], mtcnn_runtime),
// so the 32x32 path's 16 rows per lane group land on 16 distinct 4-bank slots (72-dword rows
// alone give each slot twice).  C2_SWZ: conv2's split output stores odd rows' 16 channels
// swapped the same way, so a lane group's two cell rows read disjoint slots.
constexpr int P_POOL = P_POOL0 > P_W3 + 2 * 32 * W3_ROW / 2 ? P_POOL0 : P_W3 + 2 * 32 * W3_ROW / 2;
constexpr int P_LVLH = PL_H * PL_W * 4;                // level as fp16 split planes [2][y][x][4] (in floats)
constexpr int P_A0 = P_C2 > P_LVL ? P_C2 : P_LVL;
// + 4 floats of zero padding after the split level planes: conv1's 16-byte operand reads run one
// pixel past the last level pixel (against zero weights, so the bytes there must be finite)
constexpr int P_A = P_LVLH + 4;
static_assert(P_A0 <= P_LVLH, "the level pad must lie past every other use of sA");

// exact x / k for the bin averages: power-of-two k is an exact multiply (bit-identical to the
// IEEE division), other k take the correctly-rounded division
__device__ inline float div_bin(float x, int k) {
    return (k & (k - 1)) == 0 ? x * __int_as_float((127 - __builtin_ctz(k)) << 23) : __fdiv_rn(x, (float)k);
}

// x / k for the bin averages of the downsampled levels: for k <= 3 the fma-corrected reciprocal
// q + (x - q k) y (y = RN(1/k), q = RN(x y)) equals the correctly rounded division on every
// x = s 2^-8 (|s| <= 2295, a bin of at most 9 pixels) and on every such quotient divided again
// (exhaustive check over 55k cases): 3 instructions instead of the ~10 of the IEEE
// division; larger k take the division
__device__ inline float div_small(float x, int k) {
    if (k > 3) return __fdiv_rn(x, (float)k);
    const float y = k == 3 ? __int_as_float(0x3eaaaaab) : (k == 2 ? 0.5f : 1.0f);
    const float q = x * y;
    return fmaf(fmaf(-q, (float)k, x), y, q);
}

// workgroups per CU from the LDS footprint (160 KB per CU)
constexpr int PNET_LDS = (P_A + P_POOL) * 4 + (PL_H + PL_W) * 4 + 16;

// the same split from u = 2048 v (the epilogues carry their values 2048-scaled, which is exact:
// 2048 round(c + d 2^-11) = round(2048 c + d) is one fma, and bias / PReLU commute with the
// scaling): x0 = fp16(u 2^-11) = fp16(v), x1 = fp16(u - 2048 x0) = fp16(2048 (v - x0)) -- one
// v_fma_mix each (f16 widening and the final rounding are part of the instruction).  (A zero v
// may give +0 where split_f16 gives -0: the products it feeds are zero either way.)
__device__ inline void split_u(float u, _Float16& x0, _Float16& x1) {
    x0 = (_Float16)fmaf(u, 0.00048828125f, 0.f);
    x1 = (_Float16)fmaf((float)x0, -2048.f, u);
}

// PReLU with the slope class known at compile time: slopes in [0, 1] (U) make it max(v, a v)
template <bool U>
__device__ inline float prelu_t(float v, float a) {
    return U ? fmaxf(v, a * v) : prelu(v, a);
}

// 8 halves from an 8-byte aligned LDS address as two ds_read_b64 (2 LDS cycles each, 32-lane
// bank groups over 64 banks).  The accesses are volatile so they are not merged into one
// ds_read2_b64, which costs 8 cycles (half the bandwidth) and banks over 32 dwords per 16 lanes.
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;
typedef const volatile __attribute__((address_space(3))) f16x4 lds_f16x4;
__device__ inline f16x8 ld_h8(const _Float16* p) {
    const f16x4 lo = *(lds_f16x4*)p, hi = *(lds_f16x4*)(p + 4);
    return f16x8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
}

// level pixel i of the tile: fp32 channel planes [3][PL_H*PL_W] (fp32 conv1), or fp16 split
// planes [2][PL_H*PL_W][4] (channel 3 zero) for conv1 on the matrix cores
__device__ inline void store_level(float* sA, bool split, int i, float r, float g, float b) {
    if (split) {
        _Float16 r0, r1, g0, g1, b0, b1;
        split_f16(r, r0, r1);
        split_f16(g, g0, g1);
        split_f16(b, b0, b1);
        typedef __attribute__((ext_vector_type(4))) _Float16 h4;
        h4* p = (h4*)sA;
        p[i] = h4{r0, g0, b0, (_Float16)0.f};
        p[PL_H * PL_W + i] = h4{r1, g1, b1, (_Float16)0.f};
    } else {
        sA[i] = r;
        sA[PL_H * PL_W + i] = g;
        sA[2 * PL_H * PL_W + i] = b;
    }
}

// n / d for 0 <= n < 2^31, 0 < d, quotient < 2^21 (tile indices, bin bounds): a float reciprocal
// estimate is within one of the quotient (relative error < 2^-22), corrected once each way --
// exact, in ~9 instructions instead of the ~20 of the generic 32-bit division
__device__ inline int udiv_est(int n, int d) {
    int q = (int)((float)n * __builtin_amdgcn_rcpf((float)d));
    const int r = n - q * d;
    q += r >= d ? 1 : 0;
    q -= r < 0 ? 1 : 0;
    return q;
}

// a level descriptor from the constant address space (scalar loads; the generic copy
// constructor does not take an address-space-qualified source)
__device__ inline PNetLevel load_level(const VTF_CONST PNetLevel* p) {
    PNetLevel r;
    r.lh = p->lh, r.lw = p->lw, r.ph = p->ph, r.pw = p->pw, r.scale = p->scale;
    r.tiles_x = p->tiles_x, r.tiles_y = p->tiles_y, r.pad = p->pad, r.tile_beg = p->tile_beg, r.pre = p->pre;
    return r;
}

// bytes [i0, i0 + 8) of a frame patch of w-byte rows at row stride rs, read through a buffer
// descriptor over the patch's byte extent (32-bit offsets; bytes past the extent read 0: no
// clamping), packed little-endian into two dwords.  With w >= 8 the 8 bytes span at most one row
// change: two bases and one select per byte (wave-uniform branch; narrower patches step per byte)
__device__ inline uint2 patch_bytes8(__amdgpu_buffer_rsrc_t rsrc, int i0, int w, int rs) {
    uint32_t v[2] = {0u, 0u};
    int r = udiv_est(i0, w), q = i0 - r * w;
    if (w >= 8) {
        const int o0 = r * rs + q, o1 = o0 + rs - w, k = w - q;
#pragma unroll
        for (int j = 0; j < 8; j++)
            v[j >> 2] |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rsrc, (j < k ? o0 : o1) + j, 0, 0) << (8 * (j & 3));
    } else {
#pragma unroll
        for (int j = 0; j < 8; j++) {
            v[j >> 2] |= (uint32_t)__builtin_amdgcn_raw_buffer_load_b8(rsrc, r * rs + q, 0, 0) << (8 * (j & 3));
            if (++q == w) q = 0, r++;
        }
    }
    return make_uint2(v[0], v[1]);
}

constexpr int PNET_TILE_CHUNK = 4;  // default tiles per atomic chunk (VTF_PNET_CHUNK)
constexpr int PNET_GROUPS_PER_CU = (160 * 1024) / ((PNET_LDS + 511) / 512 * 512);  // LDS granule: 512 B
static_assert(PNET_GROUPS_PER_CU >= 2, "k_pnet tile too large for 2 workgroups per CU");

// LDS plan per variant.  X (exact-levels variant, the upsampled levels that hold ~88 % of the tiles
// at min_face_size 5): the level tile is one fp16 plane (8 B per pixel, x1 = 0), so sA only has to
// hold the split conv2 output (+ the 4-float zero pad), and conv3's weights sit at the start of the
// pooled buffer (the next tile's prefetched patch is stored after a barrier instead of beside
// them): 40.4 KB -> four workgroups per CU instead of three.
template <bool X>
struct PnLds {
    static constexpr int A = X ? P_C2 + 4 : P_A;                     // floats
    static constexpr int POOL = X ? PQ_C * PP_H * PP_W : P_POOL;      // floats (split pooled conv1)
    static constexpr int W3 = X ? 0 : P_W3;                           // conv3 weights (floats)
    static constexpr int PATCH = (POOL - 4) * 4;                      // staged frame patch (bytes)
    static constexpr int BYTES = (A + POOL) * 4 + (PL_H + PL_W) * 4 + 16 + 64 + 256;  // + s_c3
    static constexpr int GPC = (160 * 1024) / ((BYTES + 511) / 512 * 512);
    static_assert(!X || (2 * P_C2 >= PL_H * PL_W * 4 + 4 && POOL >= 2 * 32 * W3_ROW / 2 && GPC >= 4),
                  "exact-levels k_pnet LDS plan");
};

// VR (vertical reuse, round 6; the exact-levels variant): a level's tiles are numbered column by
// column (ty fastest), so a workgroup's consecutive tiles are vertically adjacent.  A tile whose
// predecessor in its column was the workgroup's previous tile ("continuing") takes that tile's
// pooled conv1 rows 16..19 and conv2 rows 16, 17 as its own rows 0..3 / 0, 1 -- the same values:
// the same level pixels through the same arithmetic -- and computes only the rest: level rows
// 8..41, conv1 on pooled rows 4..19 (80 of 100 fragments), conv2 on rows 2..17 (18 of 21
// fragments).  The kept rows go through a per-workgroup slot in global memory (written after
// the tile's conv1 / conv2 with 16-byte stores, read back by LDS-DMA into rows 0..3 / 0, 1 after
// the next tile's fill / conv1), so the LDS plan is unchanged (four workgroups per CU).
constexpr int VR_POOL_BYTES = 2 * 4 * PP_W * PQ_C * 2;  // pooled rows 16..19 of both planes: 3840 B
constexpr int VR_C2_BYTES = 2 * 2 * PC_W * 16 * 2;      // conv2 rows 16, 17 of both planes: 2304 B
constexpr int VR_SLOT = VR_POOL_BYTES + VR_C2_BYTES;
constexpr int VR_LROW = 8;                              // first level row a continuing tile fills
static_assert(VR_POOL_BYTES == 3840 && VR_C2_BYTES == 2304, "VR slot pieces (the DMA piece split below)");

struct TileGeo {
    int b, ty, tx;
};
// tile t of a level -> (frame, tile row, tile column): row-major, or column-major (VR)
template <bool VR>
__device__ inline TileGeo tile_geo(int t, const PNetLevel& P) {
    const int tpi = P.tiles_x * P.tiles_y;
    const int b = udiv_est(t, tpi), tt = t - b * tpi;
    if (VR) {
        const int tx = udiv_est(tt, P.tiles_y);
        return TileGeo{b, tt - tx * P.tiles_y, tx};
    }
    const int ty = udiv_est(tt, P.tiles_x);
    return TileGeo{b, ty, tt - ty * P.tiles_x};
}

// PR: the pre-resampled variant (round 3) -- tiles of the downsampled levels, all precomputed as
// fp16 split pixels by k_resample_sat_multi, on the exact-levels LDS plan (four workgroups per CU):
// the two-plane level tile (28 KB) does not fit beside the pooled map, so conv1 runs in two halves
// of 10 pooled rows, each on 22 level rows (14.8 KB) loaded straight from the precomputed level.
template <bool DENSE, bool X, bool PR = false, bool VR = false>
__global__ __launch_bounds__(256, PnLds<X || PR>::GPC) void k_pnet(const uint8_t* __restrict__ frames, int64_t frame_stride,
                                                 int64_t row_stride, int H, int W,
                                                 const PNetLevel* __restrict__ lv, int n_levels,
                                                 int64_t total_tiles, uint32_t* __restrict__ tile_ctr, PNetW wg,
                                                 PNetOut o, int64_t tile_base, int max_chunks, int chunk) {
    using LP = PnLds<X || PR>;
    static_assert(!VR || ((X || PR) && !DENSE), "vertical reuse: the exact-levels and PR variants");
    const VTF_CONST float* wf = cptr(wg.c1w);  // fp32 weights (scalar loads at constant offsets)
    // conv / head weights through buffer loads: one lane VGPR offset + constant SGPR offsets,
    // instead of a 64-bit address per k-step (which the compiler would keep live across tiles);
    // (k rows 90, 91 of conv2 are zeroed explicitly)
    // (descriptors per tensor, built from the two bases: small constant soffsets stay immediates)
    const __amdgpu_buffer_rsrc_t rw2 = __builtin_amdgcn_make_buffer_rsrc((void*)(wg.c1w + PW_C2W), 0, 90 * 16 * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw3 = __builtin_amdgcn_make_buffer_rsrc((void*)(wg.c1w + PW_C3W), 0, 144 * 32 * 4, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw2h = __builtin_amdgcn_make_buffer_rsrc((void*)(wg.c3h + PH_C2H), 0, 2 * 16 * 96 * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t rw1h = __builtin_amdgcn_make_buffer_rsrc((void*)(wg.c3h + PH_C1H), 0, 2 * 16 * 64 * 2, 0x00020000);
    const __amdgpu_buffer_rsrc_t rhh = __builtin_amdgcn_make_buffer_rsrc((void*)(wg.c3h + PH_HH), 0, 2 * 32 * 32 * 2, 0x00020000);
    // conv3 on fp16 matrix cores (mtcnn_runtime: range bound); the X variant is launched only then
    const bool split3 = X || PR || wg.c3h != nullptr;
    __shared__ __attribute__((aligned(16))) float sA[LP::A];     // level tile, later conv2 output
    __shared__ __attribute__((aligned(16))) float sP[LP::POOL];  // frame patch (u8) during the fill, then pooled conv1
    __shared__ ushort2 ybin[PL_H], xbin[PL_W];  // frame bin [start, end) of each level row / column
    __shared__ int s_tile, s_next, s_cend;
    __shared__ unsigned long long s_clk[8];  // phase clocks (VTF_PNET_DEBUG & 256)
    // conv3 bias / PReLU slope in the 32x32 accumulator order: [bias | slope][lane half][16]
    __shared__ __attribute__((aligned(16))) float s_c3[64];
    const int tid0 = threadIdx.x, tid = tid0;
    bool pf_done = false;  // the first 2 KB of this tile's frame patch were staged by the previous tile
    int n_chunks = 0;      // chunks taken after the first (thread 0)
    int L_prev = 0;
    int64_t blk_prev = -2;  // (VR) the workgroup's previous tile
    // phase timing (debug): thread 0 reads the shader clock after each phase's closing barrier
    const bool clk_on = o.clk != nullptr;
    __shared__ unsigned long long s_tlast;  // (in LDS: a 64-bit register live across the tile loop otherwise)
    // (the uniform flag is tested first and expected off: the common path falls through instead of
    //  taking an exec-skip branch per mark)
    auto mark = [&](int k) {
        if (__builtin_expect(clk_on, 0) && tid == 0) {
            const unsigned long long t = clock64();
            s_clk[k] += t - s_tlast;
            s_tlast = t;
        }
    };
    if (tid < 8) s_clk[tid] = 0;
    if (tid == 0 && clk_on) s_tlast = clock64();
    const int lr = tid & 15;  // (the tile loop re-derives the lane coordinates per tile)

    // ---- weights and im2col offsets, loaded once per persistent workgroup
    const float b2 = wf[PW_C2B + lr], a2 = wf[PW_P2 + lr];
    // ---- tiles come from an atomic counter (dynamic: pyramid tiles differ in cost); the next
    //      index is requested as soon as the current one is known, so the atomic's round trip
    //      overlaps the tile's work instead of opening it
    // zero pad after the split level planes: read by conv1 (against zero weights) one pixel past
    // the last level pixel, and conv3's zero weight slots (k >= 144) point at it
    if (tid < 4) sA[LP::A - 4 + tid] = 0.f;
    if (tid < 64) {  // register r of lane half h holds channel (r & 3) + 8 (r >> 2) + 4 h
        const int r = tid & 15, ch = (r & 3) + 8 * (r >> 2) + 4 * ((tid >> 4) & 1);
        s_c3[tid] = tid < 32 ? wf[PW_C3B + ch] : wf[PW_P3 + ch];
    }
    // tiles are handed out in chunks of PNET_TILE_CHUNK: one same-address atomic per chunk (a
    // single counter hit once per tile serialises ~166k atomics per launch at the L2)
    if (tid == 0) {
        s_tile = (int)(tile_base + atomicAdd(tile_ctr, (uint32_t)chunk));
        s_cend = s_tile + chunk;
    }
    // (the first tile's barrier; later tiles start behind the previous tile's closing barrier)
    __syncthreads();
    for (;;) {
        mark(0);  // 0: end-of-tile prefetch store + loop barrier
        // (wave-uniform: the level table and tile geometry below become scalar loads)
        // thread coordinates laundered per tile: everything derived from them below is recomputed
        // inside the tile instead of being hoisted out of the persistent loop into long-lived
        // registers (the kernel runs at the 128-register limit of four workgroups per CU)
        int tid = tid0;
        asm volatile("" : "+v"(tid));
        const int lane = tid & 63, wave = tid >> 6;
        const int lr = lane & 15, lk = lane >> 4;
        (void)lr, (void)lk;
        const int64_t blk = __builtin_amdgcn_readfirstlane(s_tile);
        if (blk >= total_tiles) break;
        uint32_t next_tile = 0, next_cend = 0;
        if (tid == 0) {
            const int cend = s_cend;
            if (blk + 1 < cend) {
                next_tile = (uint32_t)(blk + 1);
                next_cend = (uint32_t)cend;
            } else if (max_chunks > 0 && ++n_chunks >= max_chunks) {
                // quota reached: the workgroup exits after this tile (a later workgroup of the
                // grid takes over), so its CU slot can go to other streams' kernels meanwhile
                next_tile = (uint32_t)total_tiles;
                next_cend = next_tile;
            } else {  // last tile of the chunk: request the next chunk now, used at the tile's end
                next_tile = (uint32_t)(tile_base + atomicAdd(tile_ctr, (uint32_t)chunk));
                next_cend = next_tile + chunk;
            }
            s_next = (int)next_tile;  // read after conv1 (VR) and at conv3 (prefetch)
        }
        // a workgroup's tiles come in increasing order, so its level only moves forward
        int L = L_prev;
        const VTF_CONST PNetLevel* lvc = cptr(lv);  // constant address space: scalar loads
        while (L + 1 < n_levels && blk >= lvc[L + 1].tile_beg) L++;
        const PNetLevel P = load_level(lvc + L);
        L_prev = L;
        // (tile indices are < 2^31: launch_pnet)
        const TileGeo tg = tile_geo<VR>((int)(blk - P.tile_beg), P);
        const int b = tg.b;
        const int oy0 = tg.ty * PT_H, ox0 = tg.tx * PT_W;
        // (VR) continuing tile: the previous one was the tile above it, computed by this workgroup
        const bool cont = VR && blk == blk_prev + 1 && tg.ty > 0;
        const int lr0 = cont ? VR_LROW : 0;  // first level row to fill
        blk_prev = blk;
        const uint8_t* fr = frames + (int64_t)b * frame_stride;
        const int L1h = P.lh - 2, L1w = P.lw - 2;
        // lane coordinates laundered per tile: per-lane addressing below is recomputed inside the
        // tile instead of being hoisted out of the persistent loop into long-lived registers
        int lrx = lr, lkx = lk;
        asm volatile("" : "+v"(lrx), "+v"(lkx));

        // ---- 1. level tile (rows 2*oy0 .. +42, cols 2*ox0 .. +74) = MTCNN._resample of the
        //         preprocessed frame, bit-exact; zero outside the level.
        if (tid < PL_H) {
            int ly = 2 * oy0 + tid;
            ybin[tid] = ly < P.lh ? make_ushort2(udiv_est(ly * H, P.lh), udiv_est((ly + 1) * H + P.lh - 1, P.lh))
                                  : make_ushort2(0, 0);
        } else if (tid < PL_H + PL_W) {
            int q = tid - PL_H, lx = 2 * ox0 + q;
            xbin[q] = lx < P.lw ? make_ushort2(udiv_est(lx * W, P.lw), udiv_est((lx + 1) * W + P.lw - 1, P.lw))
                                : make_ushort2(0, 0);
        }
        __syncthreads();
        mark(1);  // 1: tile index, level lookup, bins
        // frame patch covering every bin of the tile; staged to LDS with coalesced loads when it fits
        int fy0 = ybin[lr0].x, fx0 = xbin[0].x, fy1 = fy0, fx1 = fx0;
        {
            int ry = min(PL_H - 1, P.lh - 1 - 2 * oy0), rx = min(PL_W - 1, P.lw - 1 - 2 * ox0);
            fy1 = ybin[ry].y;
            fx1 = xbin[rx].y;
        }
        const int pw3 = (fx1 - fx0) * 3;
        const bool staged = !P.pre && (int64_t)(fy1 - fy0) * pw3 <= LP::PATCH;
        uint8_t* patch = (uint8_t*)sP;
        // (gathers below issue 8 loads per thread before the first use: latency-bound otherwise)
        // (nothing left to stage -- the whole patch came with the previous tile's prefetch, the
        //  common case on the upsampled levels -- needs no barrier: block-uniform condition)
        const bool stage_more = staged && !(o.dbg & 64) && (fy1 - fy0) * pw3 > (pf_done ? 256 * 8 : 0);
        if (stage_more) {
            // 8 consecutive patch bytes per thread (one 8-byte LDS store); the first 2 KB were
            // prefetched during the previous tile when pf_done
            const int nbytes = (fy1 - fy0) * pw3;
            const uint8_t* src = fr + (int64_t)fy0 * row_stride + fx0 * 3;
            const __amdgpu_buffer_rsrc_t rs_src = __builtin_amdgcn_make_buffer_rsrc(
                (void*)src, 0, (int)((fy1 - fy0 - 1) * (int)row_stride + pw3), 0x00020000);
            // four 2 KB rounds in flight per trip (the loads of a round no longer wait for the
            // previous round's stores: the downsampled levels' 7-14 KB patches were latency-bound)
            for (int i0 = 8 * tid + (pf_done ? 256 * 8 : 0); i0 < nbytes; i0 += 4 * 256 * 8) {
                uint2 pv[4];
#pragma unroll
                for (int u = 0; u < 4; u++)
                    pv[u] = i0 + u * 2048 < nbytes ? patch_bytes8(rs_src, i0 + u * 2048, pw3, (int)row_stride)
                                                   : make_uint2(0u, 0u);
#pragma unroll
                for (int u = 0; u < 4; u++)
                    if (i0 + u * 2048 < nbytes) *(uint2*)(patch + i0 + u * 2048) = pv[u];
            }
            __syncthreads();
        }
        mark(2);  // 2: frame patch staging
        if (!X && !PR && P.pre && P.pad == 1) {
            // downsampled level precomputed by k_resample_sat_multi as fp16 split pixels (12 B:
            // x0 RGB | x1 RGB, bit-identical to store_level's split of the bin average): the fill
            // is one 12-byte load and two 8-byte LDS stores per level pixel, all loads in flight
            typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
            const uint3* pre3 = (const uint3*)P.pre + (int64_t)b * P.lh * P.lw;
            u32x2* lvl = (u32x2*)sA;
            int tl = tid;
            asm volatile("" : "+v"(tl));
            const int fq = tl % PL_W, fr0 = tl < 6 * PL_W ? tl / PL_W : PL_H;
            const int lx = 2 * ox0 + fq;
            const bool inx = lx < P.lw;
            const int64_t cx = min(lx, P.lw - 1);
            uint3 v[7];
#pragma unroll
            for (int j = 0; j < 7; j++) {
                const int r = min(fr0 + 6 * j, PL_H - 1), ly = 2 * oy0 + r;
                const uint3 t = pre3[(int64_t)min(ly, P.lh - 1) * P.lw + cx];
                v[j] = inx && ly < P.lh ? t : make_uint3(0u, 0u, 0u);
            }
#pragma unroll
            for (int j = 0; j < 7; j++) {
                const int r = fr0 + 6 * j;
                if (r < PL_H) {
                    lvl[r * PL_W + fq] = u32x2{v[j].x, v[j].y & 0xffffu};
                    lvl[PL_H * PL_W + r * PL_W + fq] = u32x2{(v[j].y >> 16) | (v[j].z << 16), v[j].z >> 16};
                }
            }
        } else if (!X && !PR && P.pre) {
            // large-bin level precomputed by k_resample_sat (fp32 planes; bit-identical values).
            // (the PR variant loads its split levels inside conv1; until round 6 it also ran this
            //  fill on them -- 21 KB of misread fp32 planes per tile into LDS that conv1 then
            //  overwrote: 564 of the launch's 1,166 MB fetched, profiles/r06_pr_fetch_masks.txt)
            const float* pre = P.pre + (int64_t)b * 3 * P.lh * P.lw;
            const int64_t pl = (int64_t)P.lh * P.lw;
            for (int i0 = tid; i0 < ((o.dbg & 1) ? 0 : PL_H * PL_W); i0 += 256 * 4) {
                float v[4][3];
#pragma unroll
                for (int j = 0; j < 4; j++) {
                    const int i = min(i0 + j * 256, PL_H * PL_W - 1);
                    const int r = i / PL_W, q = i - r * PL_W;
                    const int ly = 2 * oy0 + r, lx = 2 * ox0 + q;
                    const bool in = ly < P.lh && lx < P.lw;
                    const int64_t o0 = (int64_t)min(ly, P.lh - 1) * P.lw + min(lx, P.lw - 1);
#pragma unroll
                    for (int c = 0; c < 3; c++) {
                        const float t = pre[c * pl + o0];
                        v[j][c] = in ? t : 0.f;
                    }
                }
#pragma unroll
                for (int j = 0; j < 4; j++)
                    if (i0 + j * 256 < PL_H * PL_W) store_level(sA, split3, i0 + j * 256, v[j][0], v[j][1], v[j][2]);
            }
        }
        // separable fill: the bin sums are exact integers in any order (see sat_box), so row sums
        // over each level column's bin (pass H, int16 in LDS after the patch) then column sums
        // over each level row's bin (pass V) give the reference's fp32 bin sums bit for bit, with
        // each frame byte read ~once instead of once per covering level pixel
        const int nrows = fy1 - fy0;
        const int hs_off = (nrows * pw3 + 7) & ~7;
        // upsampled levels on the split path: bins of 1 or 2 frame pixels per side, every level
        // value s * 2^-(8..10) exact in fp16 (conv1 skips the residual plane there)
        // (X: every level is exact and the host checked that its patch + row sums fit)
        const bool exact_fill = X || (!PR && split3 && P.lh >= H && P.lw >= W);
        const bool sep = staged && !(o.dbg & 1) && hs_off + nrows * PL_W * (exact_fill ? 8 : 6) <= LP::PATCH &&
                         W < 128 * P.lw;
        if (sep && exact_fill) {
            // bins of n in {0, 1, 2} pixels: branch-free sums, 8-byte row-sum entries, one store
            // per level pixel (plane 0 only; the value is its own fp16 split: x1 = 0)
            typedef __attribute__((ext_vector_type(4))) short s16x4;
            s16x4* hs = (s16x4*)(patch + hs_off);
            // 2-D thread map: column fq of every 6th row from fr0 (252 of the 256 threads), so the
            // column's bin is read and decoded once per tile instead of once per element
            // (tid laundered per tile: the map would otherwise be hoisted into long-lived registers)
            int tl = tid;
            asm volatile("" : "+v"(tl));
            const int fq = tl % PL_W, fr0 = tl < 6 * PL_W ? tl / PL_W : PL_H;
            const ushort2 xbq = xbin[fq];
            const int nq = xbq.y - xbq.x, mq = nq > 1 ? 1 : 0;
            {
                const uint8_t* col = patch + (nq ? (xbq.x - fx0) * 3 : 0);
                const uint8_t* col2 = col + 3 * mq;
                const int sub = 255 * nq;
                for (int r = fr0; r < nrows; r += 6) {
                    const uint8_t* row = col + r * pw3;
                    const uint8_t* row2 = col2 + r * pw3;
                    const int a0 = row[2] + mq * row2[2], a1 = row[1] + mq * row2[1], a2 = row[0] + mq * row2[0];
                    hs[r * PL_W + fq] = s16x4{(short)(2 * a0 - sub), (short)(2 * a1 - sub), (short)(2 * a2 - sub), 0};
                }
            }
            __syncthreads();
            typedef __attribute__((ext_vector_type(4))) _Float16 h4;
            h4* lvl = (h4*)sA;
            // conv1's operand reads run one pixel past plane 0 (against zero weights) into plane
            // 1, which this path leaves stale: that pixel must be finite
            if (tid == 0) lvl[PL_H * PL_W] = h4{(_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
            // s / kh / kw with kh, kw in {1, 2}: a power-of-two scale, exact
            const float scw = nq > 1 ? 0.001953125f : 0.00390625f;
            for (int r = fr0 + lr0; r < PL_H; r += 6) {
                const ushort2 yb = ybin[r];
                const int kh = yb.y - yb.x;
                const s16x4* h = hs + (kh ? yb.x - fy0 : 0) * PL_W + fq;
                const s16x4 v0 = h[0], v1 = h[kh > 1 ? PL_W : 0];
                const int m = kh > 1 ? 1 : 0;
                const float sc = kh > 1 ? 0.5f * scw : scw;
                const bool in = kh > 0 && nq > 0;
                const float r0 = in ? (float)(v0[0] + m * v1[0]) * sc : 0.f;
                const float g0 = in ? (float)(v0[1] + m * v1[1]) * sc : 0.f;
                const float b0 = in ? (float)(v0[2] + m * v1[2]) * sc : 0.f;
                lvl[r * PL_W + fq] = h4{(_Float16)r0, (_Float16)g0, (_Float16)b0, (_Float16)0.f};
            }
        } else if (!X && !PR && sep) {
            // downsampled levels (bins of 1-3 frame pixels per side: lh >= H / 2, the rest are
            // precomputed): the exact fill's 2-D thread map (column fq of every 6th row, the
            // column's bin decoded once) and the bin divisions by the fma-corrected reciprocal
            // (div_small: bit-identical to the correctly rounded division on this domain)
            int16_t* hs = (int16_t*)(patch + hs_off);
            int tl = tid;
            asm volatile("" : "+v"(tl));
            const int fq = tl % PL_W, fr0 = tl < 6 * PL_W ? tl / PL_W : PL_H;
            const ushort2 xbq = xbin[fq];
            const int nq = xbq.y - xbq.x;
            {
                const uint8_t* col = patch + (nq ? (xbq.x - fx0) * 3 : 0);
                for (int r = fr0; r < nrows; r += 6) {
                    const uint8_t* row = col + r * pw3;
                    int a0 = 0, a1 = 0, a2 = 0;
                    for (int x = 0; x < nq; x++) {
                        a0 += row[3 * x + 2];
                        a1 += row[3 * x + 1];
                        a2 += row[3 * x];
                    }
                    int16_t* o = hs + 3 * (r * PL_W + fq);
                    o[0] = (int16_t)(2 * a0 - 255 * nq);
                    o[1] = (int16_t)(2 * a1 - 255 * nq);
                    o[2] = (int16_t)(2 * a2 - 255 * nq);
                }
            }
            __syncthreads();
            for (int r = fr0; r < PL_H; r += 6) {
                const int ys = ybin[r].x, kh = ybin[r].y - ys;
                const int16_t* h = hs + ((kh ? ys - fy0 : 0) * PL_W + fq) * 3;
                int s0 = 0, s1 = 0, s2 = 0;
                for (int y = 0; y < kh; y++) {
                    s0 += h[y * PL_W * 3];
                    s1 += h[y * PL_W * 3 + 1];
                    s2 += h[y * PL_W * 3 + 2];
                }
                const bool in = kh > 0 && nq > 0;
                store_level(sA, split3, r * PL_W + fq, in ? div_small(div_small((float)s0 * 0.00390625f, kh), nq) : 0.f,
                            in ? div_small(div_small((float)s1 * 0.00390625f, kh), nq) : 0.f,
                            in ? div_small(div_small((float)s2 * 0.00390625f, kh), nq) : 0.f);
            }
        }
        for (int i = tid; i < (X || PR || (o.dbg & 1) || P.pre || sep ? 0 : PL_H * PL_W); i += 256) {
            int r = i / PL_W, q = i - r * PL_W;
            const int2 yb = make_int2(ybin[r].x, ybin[r].y), xb = make_int2(xbin[q].x, xbin[q].y);
            float s0 = 0.f, s1 = 0.f, s2 = 0.f;
            if (staged) {
                for (int y = yb.x; y < yb.y; y++) {
                    const uint8_t* row = patch + (y - fy0) * pw3 + (xb.x - fx0) * 3;
                    for (int x = 0; x < xb.y - xb.x; x++) {
                        s0 = s0 + ((float)row[3 * x + 2] - 127.5f) * 0.0078125f;
                        s1 = s1 + ((float)row[3 * x + 1] - 127.5f) * 0.0078125f;
                        s2 = s2 + ((float)row[3 * x] - 127.5f) * 0.0078125f;
                    }
                }
            } else {
                for (int y = yb.x; y < yb.y; y++) {
                    const uint8_t* row = fr + (int64_t)y * row_stride;
                    for (int x = xb.x; x < xb.y; x++) {
                        const uint8_t* px = row + x * 3;  // BGR
                        s0 = s0 + ((float)px[2] - 127.5f) * 0.0078125f;
                        s1 = s1 + ((float)px[1] - 127.5f) * 0.0078125f;
                        s2 = s2 + ((float)px[0] - 127.5f) * 0.0078125f;
                    }
                }
            }
            int kh = yb.y - yb.x, kw = xb.y - xb.x;
            bool in = kh > 0 && kw > 0;
            store_level(sA, split3, i, in ? div_bin(div_bin(s0, kh), kw) : 0.f, in ? div_bin(div_bin(s1, kh), kw) : 0.f,
                        in ? div_bin(div_bin(s2, kh), kw) : 0.f);
        }
        // (VR) the previous tile's slot stores (issued long before) have completed before any wave
        // of this workgroup reads the slot back
        if (VR && cont) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        mark(3);  // 3: level tile fill
        // (VR) pooled rows 0..3 <- the previous tile's rows 16..19 from the workgroup's slot: plane p
        // rows 0..3 are bytes [p 9600, p 9600 + 1920) of sP; one 1 KB LDS-DMA piece per wave (the
        // patch and row sums that used sP are dead), waited for before conv1's closing barrier
        uint8_t* vslot = VR ? o.vr + (int64_t)blockIdx.x * VR_SLOT : nullptr;
        if (VR && cont) {
            const int w = __builtin_amdgcn_readfirstlane(wave), pl = w >> 1, hf = w & 1;
            if (!hf || lane < (VR_POOL_BYTES / 2 - 1024) / 16)
                __builtin_amdgcn_global_load_lds(
                    (const void __attribute__((address_space(1)))*)(vslot + pl * (VR_POOL_BYTES / 2) + hf * 1024 + lane * 16),
                    (void __attribute__((address_space(3)))*)((uint8_t*)sP + pl * (PP_H * PP_W * PQ_C * 2) + hf * 1024), 16, 0, 0);
        }

        // ---- 2. conv1 (3->10, 3x3) + PReLU + maxpool 2x2 ceil.  Default: fp16 matrix cores on
        //         split operands (below).  fp32 fallback: the VALU -- with N = 10 output channels
        //         6/16 of an fp32 MFMA tile would be padding, so fmaf chains with the weights
        //         wave-uniform in SGPRs (scalar loads), one lane per pooled cell (its 2x2 conv1
        //         window from a 3x4x4 input patch in registers), 5 channels per wave task.
        if (split3 && !(o.dbg & 2)) {
            // conv1 on 32x32x16 fp16 matrix cores (split level planes [2][y][x][4], split weights).
            // A fragment is a 2 x 4 block of pooled cells (rows py0, py0 + 1; columns px0 .. +3):
            // A row r = cell r / 4 of the block (row-major), pool corner r % 4, i.e. conv1 position
            // (2 py + dy, 2 px + dx).  K = 3 steps (ky) of 16 slots (pixels kx 0..3 x 4 halves; kx
            // 3 and channel 3 carry zero weights); lane half hk reads pixels 2 hk, 2 hk + 1 of its
            // row.  N = 32 = [w0 | w1]: the main (x0 w0) and cross (x0 w1, + x1 w0 on residual
            // levels) products of the 16 (10 real) channels side by side, so one MFMA chain per
            // fragment covers both.  Accumulator register r of lane l is row (r & 3) + 8 (r >> 2) +
            // 4 (l >> 5) of column l & 31: registers 4q .. 4q+3 are the 4 corners of cell 2q + (l >> 5).
            // One permlane16_swap per register pair (q, q + 2) hands each half-row of lanes the
            // other half's partials of the same channel: afterwards every lane holds main and cross
            // of 2 cells (q = 0, 1 in the main lanes, q = 2, 3 in the cross lanes) and combines them
            // 2048-scaled with one fma each (split_u) -- no padding rows, no duplicated lanes.
            constexpr int NPP = PP_H * PP_W;
            constexpr int FB = PP_W / 4;              // 4-cell column blocks per row pair
            constexpr int NF1 = (PP_H / 2) * FB;      // fragments per tile
            static_assert(PP_W % 4 == 0 && PP_H % 2 == 0, "conv1 fragments are 2 x 4 pooled cells");
            typedef __attribute__((ext_vector_type(16))) float f32x16;
            const _Float16* sL = (const _Float16*)sA;
            _Float16* sQ = (_Float16*)sP;
            constexpr int PLN = PL_H * PL_W * 4;      // halves per plane
            // (lane laundered per tile, as lrx / lkx: the lane-derived offsets and the weight loads
            //  below would otherwise be hoisted out of the tile loop into long-lived registers)
            int ln = lane;
            asm volatile("" : "+v"(ln));
            const int n32 = ln & 31, hk = ln >> 5;
            // B: column n32 -> plane n32 >> 4, channel n32 & 15; k = 16 s + 8 hk .. +7
            const int woff = ((n32 >> 4) * 16 * 64 + (n32 & 15) * 64 + 8 * hk) * 2;
            f16x8 wb[3];
#pragma unroll
            for (int s = 0; s < 3; s++)
                wb[s] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(rw1h, woff, 32 * s, 0));
            // bias 2048-scaled (exact): the epilogue works on u = 2048 v (split_u)
            const float b1s = lrx < 10 ? wf[PW_C1B + lrx] * 2048.f : 0.f, a1 = lrx < 10 ? wf[PW_P1 + lrx] : 0.f;
            // the tile's conv1 window lies inside the level: no per-corner bounds checks
            const bool interior = 2 * (oy0 + PP_H - 1) + 1 < L1h && 2 * (ox0 + PP_W - 1) + 1 < L1w;
            // pool-then-activate is exact when every channel's slope is >= 0 (PReLU and rounding
            // monotone); with slopes in [0, 1] PReLU is max(v, a v) (two instructions)
            const uint64_t all = ~0ull;
            const bool mono = __ballot(a1 >= 0.f) == all;
            const bool unit_slope = __ballot(a1 >= 0.f && a1 <= 1.f) == all;
            const bool fastpool = interior && mono;
            // upsampled levels (lh >= H, lw >= W: every bin 1 or 2 frame pixels per side) hold
            // s / 2^(8..10) with |s| <= 1020, exact in fp16: the residual plane is zero there, so
            // its MFMAs and operand reads are skipped (the products they would add are all zero)
            const bool exact = X || (!PR && P.lh >= H && P.lw >= W);
            const int wv = __builtin_amdgcn_readfirstlane(wave);
            // the lane's A row: cell cq of the block, corner
            const int r32 = ln & 31, cq = r32 >> 2, corner = r32 & 3;
            const int lpix = (2 * (cq >> 2) + (corner >> 1)) * PL_W + 2 * (cq & 3) + (corner & 1) + 2 * hk;
            // the cells this lane ends with: 2 q + 4 ((lane >> 4) & 1) + (lane >> 5), q = 0, 1
            const int cbase = 4 * ((ln >> 4) & 1) + (ln >> 5);
            // pooled-map slot of the lane's channel (lanes 12..15 repeat channels 10, 11, which
            // conv2 never reads)
            const int qch = lrx < 12 ? lrx : 10 + (lrx & 1);
            // residual-level cross operand [0 | w0] (general variant only)
            f16x8 wx[3] = {};
            if (!exact) {
#pragma unroll
                for (int s = 0; s < 3; s++) {
                    const f16x8 w = __builtin_bit_cast(
                        f16x8, __builtin_amdgcn_raw_buffer_load_b128(rw1h, ((n32 & 15) * 64 + 8 * hk) * 2, 32 * s, 0));
                    wx[s] = n32 >= 16 ? w : f16x8{};
                }
            }
            // NU fragments per iteration (wave-strided: F = wv + 4 k); whole iterations first,
            // then the remaining fragment one at a time.  FP: fastpool && unit_slope, a
            // compile-time branch (uniform flags tested per fragment cost a branch each)
            // fragments [f0, f_end) of the level tile in sL whose first row is level row lrow0 of the
            // tile (PR: a half tile of 22 rows, planes pln halves apart)
            int f_end = NF1, lrow0 = 0, pln = PLN;
            auto conv1_frags = [&](auto exact_t, auto fp_t, auto nu_t, int f0) -> int {
                constexpr bool EX = decltype(exact_t)::value;
                constexpr bool FP = decltype(fp_t)::value;
                constexpr int NU = decltype(nu_t)::value;
                for (; f0 + 4 * (NU - 1) < f_end; f0 += 4 * NU) {
                    int fo[NU], py0[NU], px0[NU];
#pragma unroll
                    for (int u = 0; u < NU; u++) {
                        const int f = f0 + 4 * u;
                        const int br = f / FB;
                        py0[u] = 2 * br;
                        px0[u] = 4 * (f - br * FB);
                        fo[u] = (lpix + (2 * py0[u] - lrow0) * PL_W + 2 * px0[u]) * 4;
                    }
                    f16x8 xa[3][NU], xb[3][NU];
#pragma unroll
                    for (int s = 0; s < 3; s++)
#pragma unroll
                        for (int u = 0; u < NU; u++) {
                            xa[s][u] = ld_h8(sL + fo[u] + s * PL_W * 4);
                            if (!EX) xb[s][u] = ld_h8(sL + pln + fo[u] + s * PL_W * 4);
                        }
                    f32x16 acc[NU];
#pragma unroll
                    for (int u = 0; u < NU; u++) acc[u] = f32x16{};
#pragma unroll
                    for (int s = 0; s < 3; s++)
#pragma unroll
                        for (int u = 0; u < NU; u++) {
                            acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xa[s][u], wb[s], acc[u], 0, 0, 0);
                            if (!EX) acc[u] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xb[s][u], wx[s], acc[u], 0, 0, 0);
                        }
#pragma unroll
                    for (int u = 0; u < NU; u++) {
                        float uv[2][4];  // 2048-scaled combined corners of the lane's 2 cells
#pragma unroll
                        for (int q = 0; q < 2; q++)
#pragma unroll
                            for (int i = 0; i < 4; i++) {
                                const auto sw = __builtin_amdgcn_permlane16_swap(
                                    __float_as_uint(acc[u][4 * q + i]), __float_as_uint(acc[u][4 * (q + 2) + i]), false, false);
                                uv[q][i] = fmaf(__uint_as_float(sw[0]), 2048.f, __uint_as_float(sw[1]));
                            }
#pragma unroll
                        for (int q = 0; q < 2; q++) {
                            const int c = 2 * q + cbase;
                            const int py = py0[u] + (c >> 2), px = px0[u] + (c & 3);
                            float out;
                            if (FP) {
                                const float v = fmaxf(fmaxf(uv[q][0], uv[q][1]), fmaxf(uv[q][2], uv[q][3])) + b1s;
                                out = fmaxf(v, a1 * v);
                            } else if (fastpool) {
                                out = prelu(fmaxf(fmaxf(uv[q][0], uv[q][1]), fmaxf(uv[q][2], uv[q][3])) + b1s, a1);
                            } else {
                                const int gy = 2 * (oy0 + py), gx = 2 * (ox0 + px);
                                float m = -3.402823466e38f;
                                bool any = false;
#pragma unroll
                                for (int i = 0; i < 4; i++) {
                                    const bool ok = (gy + (i >> 1) < L1h) && (gx + (i & 1) < L1w);
                                    const float v = prelu(uv[q][i] + b1s, a1);
                                    if (ok) {
                                        m = fmaxf(m, v);
                                        any = true;
                                    }
                                }
                                out = any ? m : 0.f;  // outside the valid pooled map: keep finite
                            }
                            _Float16 x0, x1;
                            split_u(out, x0, x1);
                            _Float16* qp = sQ + (py * PP_W + px) * PQ_C + qch;
                            qp[0] = x0;
                            qp[NPP * PQ_C] = x1;
                        }
                    }
                }
                return f0;
            };
            using I1 = std::integral_constant<int, 1>;
            using I2 = std::integral_constant<int, 2>;
            using T = std::true_type;
            using F = std::false_type;
            // (the boundary / general-slope epilogue runs one fragment at a time: its per-corner
            //  bounds logic would otherwise set the kernel's register peak for ~3 % of the tiles)
            if (PR) {
                // two halves: level rows [20 h, 20 h + 22) of both split planes (12-byte pixels of
                // the precomputed level, one load each, all in flight), then the 25 fragments of
                // pooled rows [10 h, 10 h + 10)
                typedef __attribute__((ext_vector_type(2))) uint32_t u32x2;
                constexpr int HR = PL_H / 2 + 1;  // 22 level rows per half
                static_assert(2 * HR * PL_W * 8 + 8 <= LP::A * 4, "PR half tile fits the level buffer");
                const uint3* pre3 = (const uint3*)P.pre + (int64_t)b * P.lh * P.lw;
                u32x2* lvl = (u32x2*)sA;
                int tl = tid;
                asm volatile("" : "+v"(tl));
                const int fq = tl % PL_W, fr0 = tl < 6 * PL_W ? tl / PL_W : HR;
                const int lx = 2 * ox0 + fq;
                const bool inx = lx < P.lw;
                const int64_t cx = min(lx, P.lw - 1);
                pln = HR * PL_W * 4;
                for (int h = 0; h < 2; h++) {
                    if (h) __syncthreads();  // the first half's fragments have read sA
                    // (VR) a continuing tile's first half: level rows 8..21 for pooled rows 4..9
                    const int rb = h == 0 ? lr0 : 0;
                    uint3 v[4];
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int r = min(rb + fr0 + 6 * j, HR - 1), ly = 2 * oy0 + 20 * h + r;
                        const uint3 t = pre3[(int64_t)min(ly, P.lh - 1) * P.lw + cx];
                        v[j] = inx && ly < P.lh ? t : make_uint3(0u, 0u, 0u);
                    }
#pragma unroll
                    for (int j = 0; j < 4; j++) {
                        const int r = rb + fr0 + 6 * j;
                        if (r < HR) {
                            lvl[r * PL_W + fq] = u32x2{v[j].x, v[j].y & 0xffffu};
                            lvl[HR * PL_W + r * PL_W + fq] = u32x2{(v[j].y >> 16) | (v[j].z << 16), v[j].z >> 16};
                        }
                    }
                    // conv1's operand reads run one pixel past plane 1 (against zero weights)
                    if (tid == 0) lvl[2 * HR * PL_W] = u32x2{0u, 0u};
                    __syncthreads();
                    f_end = NF1 / 2 * (h + 1);
                    lrow0 = 20 * h;
                    const int f0 = NF1 / 2 * h + wv + (h == 0 && cont ? 2 * FB : 0);  // (VR) pooled rows 4..
                    if (fastpool && unit_slope)
                        conv1_frags(F{}, T{}, I1{}, conv1_frags(F{}, T{}, I2{}, f0));
                    else
                        conv1_frags(F{}, F{}, I1{}, f0);
                }
            } else if (X && wg.c1k) {
                // exact levels (x1 = 0) on v_mfma_f32_16x16x32_f16, the main and cross products in
                // ONE chain: A row = (cell, corner) of a 1 x 4 run of pooled cells (lane & 15 ->
                // cell (lane & 15) >> 2, corner lane & 3), K = 3 steps x 4 lane groups of pixel pairs
                // (kx 0,1 | 2,3 of tap row ky; 4 halves a pixel): pairs 0..5 = (ky, kx pair) against
                // 2^11 w0, pairs 6..11 the same pixels against w1, so the accumulator is u = 2048 v
                // directly (the 32x32 layout needs a lane swap + fma per corner to combine its [w0 |
                // w1] columns).  The D layout hands each lane the 4 corners of one cell (lane >> 4) for
                // one channel (lane & 15): the max-pool is in-register.
                constexpr int FB4 = PP_W / 4, NF4 = PP_H * FB4;
                static_assert(PP_W % 4 == 0, "conv1 runs of 4 pooled cells");
                const int g4 = ln >> 4, r16 = ln & 15, crn = r16 & 3;
                const int abase = ((crn >> 1) * PL_W + 2 * (r16 >> 2) + (crn & 1)) * 4;
                int ko[3];
                f16x8 wk[3];
#pragma unroll
                for (int s = 0; s < 3; s++) {
                    const int i = 4 * s + g4, q = i < 6 ? i : i - 6;
                    ko[s] = ((q >> 1) * PL_W + 2 * (q & 1)) * 4;
                    const f16x8 w = __builtin_bit_cast(
                        f16x8, __builtin_amdgcn_raw_buffer_load_b128(rw1h, ((r16 + (i < 6 ? 0 : 16)) * 64 + (q >> 1) * 16 + (q & 1) * 8) * 2, 0, 0));
                    wk[s] = i < 6 ? w * (_Float16)2048.f : w;
                }
                const int cq = ln >> 4;  // the D cell of this lane
                auto c1k_frags = [&](auto fp_t, auto nu_t, int f0) -> int {
                    constexpr bool FP = decltype(fp_t)::value;
                    constexpr int NU = decltype(nu_t)::value;
                    for (; f0 + 4 * (NU - 1) < NF4; f0 += 4 * NU) {
                        int py[NU], px0[NU];
                        f16x8 xa[3][NU];
#pragma unroll
                        for (int u = 0; u < NU; u++) {
                            const int f = f0 + 4 * u, r = f / FB4;
                            py[u] = r;
                            px0[u] = 4 * (f - r * FB4);
                            const int fo = (2 * r * PL_W + 2 * px0[u]) * 4 + abase;
#pragma unroll
                            for (int s = 0; s < 3; s++) xa[s][u] = ld_h8(sL + fo + ko[s]);
                        }
                        f32x4 acc[NU];
#pragma unroll
                        for (int u = 0; u < NU; u++) acc[u] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
                        for (int s = 0; s < 3; s++)
#pragma unroll
                            for (int u = 0; u < NU; u++)
                                acc[u] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa[s][u], wk[s], acc[u], 0, 0, 0);
#pragma unroll
                        for (int u = 0; u < NU; u++) {
                            const int px = px0[u] + cq;
                            float out;
                            if (FP) {
                                const float v = fmaxf(fmaxf(acc[u][0], acc[u][1]), fmaxf(acc[u][2], acc[u][3])) + b1s;
                                out = fmaxf(v, a1 * v);
                            } else if (fastpool) {
                                out = prelu(fmaxf(fmaxf(acc[u][0], acc[u][1]), fmaxf(acc[u][2], acc[u][3])) + b1s, a1);
                            } else {
                                const int gy = 2 * (oy0 + py[u]), gx = 2 * (ox0 + px);
                                float m = -3.402823466e38f;
                                bool any = false;
#pragma unroll
                                for (int i = 0; i < 4; i++) {
                                    const bool ok = (gy + (i >> 1) < L1h) && (gx + (i & 1) < L1w);
                                    const float v = prelu(acc[u][i] + b1s, a1);
                                    if (ok) {
                                        m = fmaxf(m, v);
                                        any = true;
                                    }
                                }
                                out = any ? m : 0.f;  // outside the valid pooled map: keep finite
                            }
                            _Float16 x0, x1;
                            split_u(out, x0, x1);
                            if (r16 < PQ_C) {
                                _Float16* qp = sQ + (py[u] * PP_W + px) * PQ_C + r16;
                                qp[0] = x0;
                                qp[NPP * PQ_C] = x1;
                            }
                        }
                    }
                    return f0;
                };
                using I4 = std::integral_constant<int, 4>;
                const int f0 = wv + (cont ? 4 * FB4 : 0);  // (VR) continuing tile: pooled rows 4..19
                if (fastpool && unit_slope)
                    c1k_frags(T{}, I1{}, c1k_frags(T{}, I4{}, f0));
                else
                    c1k_frags(F{}, I1{}, c1k_frags(F{}, I2{}, f0));
            } else if (exact) {
                if (fastpool && unit_slope)
                    conv1_frags(T{}, T{}, I1{}, conv1_frags(T{}, T{}, I2{}, wv));
                else
                    conv1_frags(T{}, F{}, I1{}, wv);
            } else {
                if (fastpool && unit_slope)
                    conv1_frags(F{}, T{}, I1{}, conv1_frags(F{}, T{}, I2{}, wv));
                else
                    conv1_frags(F{}, F{}, I1{}, wv);
            }
        }
        {
            constexpr int NPP = PP_H * PP_W;        // pooled cells
            constexpr int NCH = (NPP + 63) / 64;    // 64-cell chunks
            constexpr int CG = 5;                   // channels per wave task
            constexpr int NWT = (10 / CG) * NCH;    // wave tasks
            // the tile's conv1 window lies inside the level: no per-corner bounds checks
            const bool interior = 2 * (oy0 + PP_H - 1) + 1 < L1h && 2 * (ox0 + PP_W - 1) + 1 < L1w;
            const int wv = __builtin_amdgcn_readfirstlane(wave);
            // (guarded, not only bounded: the compiler cannot prove wv >= 0, so a zero bound alone
            //  keeps the fallback's code -- and its register demand -- in the exact variant)
            for (int wt = wv; !X && !PR && wt < ((o.dbg & 2) || split3 ? 0 : NWT); wt += 4) {
                const int g = wt / NCH, chunk = wt - g * NCH;
                const bool live = chunk * 64 + lane < NPP;
                const int pp = min(chunk * 64 + lane, NPP - 1);
                const int py = pp / PP_W, px = pp - py * PP_W;
                const float* src = sA + (2 * py) * PL_W + 2 * px;
                float x[3][4][4];
#pragma unroll
                for (int c = 0; c < 3; c++)
#pragma unroll
                    for (int r = 0; r < 4; r++)
#pragma unroll
                        for (int q = 0; q < 4; q++) x[c][r][q] = src[c * PL_H * PL_W + r * PL_W + q];
                const int gy = 2 * (oy0 + py), gx = 2 * (ox0 + px);
#pragma unroll
                for (int j = 0; j < CG; j++) {
                    const int co = g * CG + j;
                    float acc[4] = {0.f, 0.f, 0.f, 0.f};  // corners (dy, dx) = (0,0) (0,1) (1,0) (1,1)
#pragma unroll
                    for (int c = 0; c < 3; c++)
#pragma unroll
                        for (int ky = 0; ky < 3; ky++)
#pragma unroll
                            for (int kx = 0; kx < 3; kx++) {
                                const float w = wf[PW_C1W + co * 27 + (c * 3 + ky) * 3 + kx];  // [co][ci][ky][kx]
                                acc[0] = fmaf(x[c][ky][kx], w, acc[0]);
                                acc[1] = fmaf(x[c][ky][kx + 1], w, acc[1]);
                                acc[2] = fmaf(x[c][ky + 1][kx], w, acc[2]);
                                acc[3] = fmaf(x[c][ky + 1][kx + 1], w, acc[3]);
                            }
                    const float bb = wf[PW_C1B + co], aa = wf[PW_P1 + co];
                    float out;
                    if (interior && aa >= 0.f) {
                        // PReLU with a non-negative slope is monotone, so max(prelu(v)) ==
                        // prelu(max(v)) bit for bit (rounding is monotone too): pool, then activate
                        out = prelu(fmaxf(fmaxf(acc[0], acc[1]), fmaxf(acc[2], acc[3])) + bb, aa);
                    } else {
                        float m = -3.402823466e38f;
                        bool any = false;
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            const bool ok = (gy + (i >> 1) < L1h) && (gx + (i & 1) < L1w);
                            const float v = prelu(acc[i] + bb, aa);
                            if (ok) {
                                m = fmaxf(m, v);
                                any = true;
                            }
                        }
                        // outside the valid pooled map (only feeds discarded cells): keep finite
                        out = any ? m : 0.f;
                    }
                    if (live) sP[co * NPP + pp] = out;
                }
            }
        }
        if (VR && cont) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the pooled rows' LDS-DMA
        __syncthreads();
        mark(4);  // 4: conv1 + pool
        // (VR) does the next tile continue this one (the tile below it, next in this workgroup)?
        const bool vr_next = VR && __builtin_amdgcn_readfirstlane(s_next) == blk + 1 && tg.ty + 1 < P.tiles_y;
        if (VR && vr_next && tid < VR_POOL_BYTES / 16) {
            // pooled rows 16..19 of both planes -> the slot (read again after the next tile's fill)
            const int pl = tid / (VR_POOL_BYTES / 32), q = tid - pl * (VR_POOL_BYTES / 32);
            const uint4 v = *(const uint4*)((const uint8_t*)sP + pl * (PP_H * PP_W * PQ_C * 2) + 16 * PP_W * PQ_C * 2 + q * 16);
            *(uint4*)(vslot + tid * 16) = v;
        }
        if (VR && cont) {
            // conv2 rows 0, 1 <- the previous tile's rows 16, 17 (plane p rows 0, 1 = sA bytes [p 10368,
            // + 1152)); the level tile there is dead after conv1's barrier; waited for before conv2's
            const int w = __builtin_amdgcn_readfirstlane(wave), pl = w >> 1, hf = w & 1;
            if (!hf || lane < (VR_C2_BYTES / 2 - 1024) / 16)
                __builtin_amdgcn_global_load_lds(
                    (const void __attribute__((address_space(1)))*)(vslot + VR_POOL_BYTES + pl * (VR_C2_BYTES / 2) + hf * 1024 + lane * 16),
                    (void __attribute__((address_space(3)))*)((uint8_t*)sA + pl * (PC_H * PC_W * 32) + hf * 1024), 16, 0, 0);
        }

        // ---- 3. conv2 (10->16, 3x3) + PReLU on MFMA: 18 x 18 positions (21 frags of 16), 16
        //         output channels, K = 90; operands gathered from the pooled map.
        {
            constexpr int NPOS = PC_H * PC_W;      // 324
            constexpr int NF = (NPOS + 15) / 16;   // 21
            if (split3 && !(o.dbg & 4)) {
                // fp16 matrix cores on split operands (as conv3), computed TRANSPOSED (rows = the 16
                // output channels, A = weights; columns = 16 conv2 positions, B = the pooled map), K =
                // 90 packed into 3 steps of 32: step 0 / 1 = channels 0-7 of taps g / 4 + g for lane
                // group g (one 16-byte read per plane); step 2 = 4 dwords per lane: group 0 channels
                // 0-7 of tap 8, groups 1 / 2 channels 8, 9 of taps 0-3 / 4-7, group 3 channels 8, 9
                // of tap 8 (+ 3 zero-weight slots).  Each lane ends with 4 consecutive output channels
                // of one position: one 8-byte store per plane.  Main and 2^11-scaled cross products
                // in separate accumulators.
                constexpr int NPP = PP_H * PP_W;
                const _Float16* sH = (const _Float16*)sP;
                typedef const volatile __attribute__((address_space(3))) uint32_t lds_u32;
                f16x8 w0[3], w1[3];
                const int woff = (lrx * 96 + 8 * lkx) * 2;
#pragma unroll
                for (int s3 = 0; s3 < 3; s3++) {
                    w0[s3] = __builtin_bit_cast(f16x8, __builtin_amdgcn_raw_buffer_load_b128(rw2h, woff, 64 * s3, 0));
                    w1[s3] = __builtin_bit_cast(f16x8,
                                                __builtin_amdgcn_raw_buffer_load_b128(rw2h, woff, 16 * 96 * 2 + 64 * s3, 0));
                }
                // operand offsets (halves) relative to the position's pooled cell
                auto tapoff = [](int t) { return ((t / 3) * PP_W + t % 3) * PQ_C; };
                const int o0 = tapoff(lkx), o1 = tapoff(4 + lkx);
                int o2[4];
#pragma unroll
                for (int jj = 0; jj < 4; jj++)
                    o2[jj] = lkx == 0 ? tapoff(8) + 2 * jj : lkx == 3 ? tapoff(8) + 8 : tapoff(4 * (lkx - 1) + jj) + 8;
                float bb[4], aa[4];  // bias 2048-scaled (split_u)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    bb[i] = wf[PW_C2B + 4 * lkx + i] * 2048.f;
                    aa[i] = wf[PW_P2 + 4 * lkx + i];
                }
                _Float16* sO = (_Float16*)sA;
                // (VR) continuing tile: rows 2..17 only (positions 36.., 18 fragments)
                const int pb = cont ? 2 * PC_W : 0, nf = cont ? (NPOS - 2 * PC_W) / 16 : NF;
                static_assert((NPOS - 2 * PC_W) % 16 == 0, "continuing-tile conv2 fragments");
                auto conv2_frags = [&](auto u_t) {
                constexpr bool U2 = decltype(u_t)::value;
                // (wave index through readfirstlane: `two` is then a scalar branch, not an exec mask)
                for (int f0 = __builtin_amdgcn_readfirstlane(wave); f0 < nf; f0 += 8) {
                    const int f1 = f0 + 4;
                    const bool two = f1 < nf;
                    const int p0 = min(pb + f0 * 16 + lrx, NPOS - 1), p1 = min(pb + (two ? f1 : f0) * 16 + lrx, NPOS - 1);
                    const int ab0 = ((p0 / PC_W) * PP_W + (p0 % PC_W)) * PQ_C, ab1 = ((p1 / PC_W) * PP_W + (p1 % PC_W)) * PQ_C;
                    f16x8 x[3][2][2];  // [step][fragment][plane]
#pragma unroll
                    for (int pl = 0; pl < 2; pl++) {
                        const _Float16* base = sH + pl * NPP * PQ_C;
                        x[0][0][pl] = ld_h8(base + ab0 + o0);
                        x[0][1][pl] = ld_h8(base + ab1 + o0);
                        x[1][0][pl] = ld_h8(base + ab0 + o1);
                        x[1][1][pl] = ld_h8(base + ab1 + o1);
                        uint32_t u0[4], u1[4];
#pragma unroll
                        for (int jj = 0; jj < 4; jj++) {
                            u0[jj] = *(lds_u32*)(base + ab0 + o2[jj]);
                            u1[jj] = *(lds_u32*)(base + ab1 + o2[jj]);
                        }
                        x[2][0][pl] = __builtin_bit_cast(f16x8, u0);
                        x[2][1][pl] = __builtin_bit_cast(f16x8, u1);
                    }
                    f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, d0 = c0, d1 = c0;
                    if (two) {
#pragma unroll
                        for (int s3 = 0; s3 < 3; s3++) {
                            c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0[s3], x[s3][0][0], c0, 0, 0, 0);
                            d0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[s3], x[s3][0][0], d0, 0, 0, 0);
                            d0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0[s3], x[s3][0][1], d0, 0, 0, 0);
                            c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0[s3], x[s3][1][0], c1, 0, 0, 0);
                            d1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[s3], x[s3][1][0], d1, 0, 0, 0);
                            d1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0[s3], x[s3][1][1], d1, 0, 0, 0);
                        }
                    } else {  // the wave's last fragment has no partner (wave-uniform): one chain pair
#pragma unroll
                        for (int s3 = 0; s3 < 3; s3++) {
                            c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0[s3], x[s3][0][0], c0, 0, 0, 0);
                            d0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[s3], x[s3][0][0], d0, 0, 0, 0);
                            d0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0[s3], x[s3][0][1], d0, 0, 0, 0);
                        }
                    }
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        const int q = pb + (h ? f1 : f0) * 16 + lrx;
                        if (q < NPOS && (h == 0 || two)) {
                            f16x4 v0, v1;
#pragma unroll
                            for (int i = 0; i < 4; i++) {
                                const float u = h ? fmaf(c1[i], 2048.f, d1[i]) : fmaf(c0[i], 2048.f, d0[i]);
                                _Float16 x0, x1;
                                split_u(prelu_t<U2>(u + bb[i], aa[i]), x0, x1);
                                v0[i] = x0;
                                v1[i] = x1;
                            }
                            // (odd rows: channel halves swapped, see C2_SWZ)
                            const int qo = q * 16 + ((4 * lkx) ^ (8 * ((q / PC_W) & 1)));
                            *(f16x4*)(sO + qo) = v0;
                            *(f16x4*)(sO + NPOS * 16 + qo) = v1;
                        }
                    }
                }
                };
                if (wg.unit_slopes & 1)
                    conv2_frags(std::true_type{});
                else
                    conv2_frags(std::false_type{});
            }
            // fp32 fallback (conv2 on fp32 MFMA): weights per tile (L1-resident), keeping the
            // persistent register set small; issued only when this path runs
            const bool fp32_conv2 = !X && !split3 && !(o.dbg & 4);
            float w2[23] = {};
            if (fp32_conv2) {
                const int w2off = (16 * lkx + lrx) * 4;
#pragma unroll
                for (int s = 0; s < 23; s++)
                    w2[s] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rw2, w2off, 256 * s, 0));
                if (lkx >= 2) w2[22] = 0.f;  // k = 90, 91: zero padding
            }
            for (int f0 = wave; fp32_conv2 && f0 < NF; f0 += 8) {
                const int f1 = f0 + 4;
                const bool two = f1 < NF;
                int p0 = min(f0 * 16 + lrx, NPOS - 1), p1 = min((two ? f1 : f0) * 16 + lrx, NPOS - 1);
                const int ab0 = (p0 / PC_W) * PP_W + (p0 % PC_W), ab1 = (p1 / PC_W) * PP_W + (p1 % PC_W);
                f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
                // operands of a whole group of k-steps are read before its MFMAs (LDS latency
                // overlapped instead of one wait per MFMA)
#pragma unroll
                for (int g = 0; g < 23; g += 12) {
                    float av0[12], av1[12];
#pragma unroll
                    for (int s = g; s < min(g + 12, 23); s++) {
                        const int k = min(4 * s + lkx, 89);
                        const int c = k / 9, r = k - 9 * c;
                        const int ko = c * PP_H * PP_W + (r / 3) * PP_W + (r % 3);
                        av0[s - g] = sP[ab0 + ko];
                        av1[s - g] = sP[ab1 + ko];
                    }
                    __builtin_amdgcn_sched_barrier(0);  // keep the reads ahead of the MFMAs
#pragma unroll
                    for (int s = g; s < min(g + 12, 23); s++) {
                        c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av0[s - g], w2[s], c0, 0, 0, 0);
                        c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av1[s - g], w2[s], c1, 0, 0, 0);
                    }
                }
                if (split3) {
                    // fp16 split planes [2][pos][16 ch]: v = x0 + x1 * 2^-11 (x0 = fp16(v), x1 =
                    // fp16((v - x0) * 2^11), the residual exact in fp32)
                    _Float16* sH = (_Float16*)sA;
#pragma unroll
                    for (int i = 0; i < 4; i++) {
#pragma unroll
                        for (int h = 0; h < 2; h++) {
                            const int q = (h ? f1 : f0) * 16 + 4 * lkx + i;
                            if (q < NPOS && (h == 0 || two)) {
                                const float v = prelu((h ? c1[i] : c0[i]) + b2, a2);
                                const _Float16 x0 = (_Float16)v;
                                sH[q * 16 + lrx] = x0;
                                sH[NPOS * 16 + q * 16 + lrx] = (_Float16)((v - (float)x0) * 2048.f);
                            }
                        }
                    }
                } else {
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        int q0 = f0 * 16 + 4 * lkx + i;
                        if (q0 < NPOS) sA[lrx * NPOS + q0] = prelu(c0[i] + b2, a2);
                        int q1 = f1 * 16 + 4 * lkx + i;
                        if (two && q1 < NPOS) sA[lrx * NPOS + q1] = prelu(c1[i] + b2, a2);
                    }
                }
            }
        }
        if (VR && cont) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // conv2 rows 0, 1 (LDS-DMA)
        __syncthreads();
        if (VR && vr_next && tid < VR_C2_BYTES / 16) {
            // conv2 rows 16, 17 of both planes -> the slot (conv3 only reads sA from here on)
            const int pl = tid / (VR_C2_BYTES / 32), q = tid - pl * (VR_C2_BYTES / 32);
            const uint4 v = *(const uint4*)((const uint8_t*)sA + pl * (PC_H * PC_W * 32) + 16 * PC_W * 32 + q * 16);
            *(uint4*)(vslot + VR_POOL_BYTES + tid * 16) = v;
        }
        if (split3) {
            // conv3's split weights [2][32][144] halves (18 KB, L2-resident) -> the pooled buffer,
            // now free: 18 lane-linear 1 KB LDS-DMA pieces, waited for by the barrier
            constexpr int W3_PIECES = 2 * 32 * W3_ROW * 2 / 1024;
            static_assert(2 * 32 * W3_ROW * 2 % 1024 == 0, "whole 1 KB pieces");
            const char* src = (const char*)wg.c3h;
            for (int c = wave; c < W3_PIECES; c += 4)
                __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(src + c * 1024 + lane * 16),
                                                 (void __attribute__((address_space(3)))*)(sP + LP::W3 + c * 256), 16, 0, 0);
            __syncthreads();
        }
        mark(5);  // 5: conv2

        // ---- 4. conv3 (16->32, 3x3) + PReLU on MFMA, computed TRANSPOSED (C = W3^T x im2col:
        //         rows = 32 channels in 2 frags, cols = 16 cells per frag, K = 144 in 36 steps) so
        //         the 1x1 heads are one more MFMA chain summing over the accumulator rows with no
        //         lane movement: Heads^T (16 x cells) = Wh^T (16 x 32) x F (32 x cells), the
        //         k-slot of lane group g at step i being channel 16*mf + 4g + i.
        //         Default path: fp16 matrix cores on split operands (x = x0 + x1 * 2^-11 from
        //         conv2's epilogue, w = w0 + w1 * 2^-11 prepared on the host): x0 w0 + 2^-11 (x0 w1 +
        //         x1 w0) is exact to ~2^-24 relative (the dropped x1 w1 is below that), 3 MFMAs of
        //         16x16x32 per 32-deep k-step instead of 8 fp32 16x16x4 ones (2.7x less matrix
        //         time).  Fallback (conv2 activations could leave the fp16 range, host bound):
        //         fp32 MFMA with the weights streamed in 4 chunks of 9 k-steps.
        // ---- next tile's frame patch: the first 8 bytes per thread (2 KB, the whole patch of the
        //      upsampled levels that dominate the tile count) are loaded at conv3's start, in
        //      flight during conv3 (which reads its weights from LDS: no later global load waits
        //      on them), and stored to the patch buffer after it -- the next tile's staging
        //      latency hides behind this tile's matrix work
        uint2 pfv = make_uint2(0u, 0u);  // the prefetched bytes 8 tid .. +7, packed
        int pf_n = 0;
        {
            constexpr int FPW = PT_H * PT_W / 64;  // 16-cell fragments per wave
            // two passes of FPW/2 fragments each: conv3 + heads per pass keeps the accumulators
            // (main + correction on the fp16 path) within the 3-workgroup register budget
            constexpr int NHALF = FPW % 2 == 0 ? 2 : 1;
            constexpr int FH = FPW / NHALF;
            // accumulator row (mf, lkx, i) = channel 16*mf + 4*lkx + i
            float cb3[2][4], ca3[2][4], hwA[2][4];
#pragma unroll
            for (int mf = 0; mf < 2; mf++)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int ch = 16 * mf + 4 * lkx + i;
                    cb3[mf][i] = wf[PW_C3B + ch] * 2048.f;  // 2048-scaled, as the accumulators
                    ca3[mf][i] = wf[PW_P3 + ch];
                    // heads as the A operand: row = head lrx (0,1 conv4_1; 2..5 conv4_2), k-slot = ch
                    const int hrow = lrx < 2 ? lrx * 32 + ch : (lrx < 6 ? (lrx - 2) * 32 + ch : 0);
                    const float hv = lrx < 2 ? wf[PW_C41W + hrow] : wf[PW_C42W + hrow];
                    hwA[mf][i] = !X && lrx < 6 ? hv : 0.f;
                }
            // split conv3 + split heads (every X launch; the general variant when the host bounds
            // hold): conv3 and the heads on 32x32x16 matrix cores (below); otherwise the 16x16
            // fallbacks (fp32 conv3 and / or fp32 heads)
            const bool splith = X || PR || wg.hh != nullptr;  // (X, PR: launched only with the split heads)
            const bool c3_32 = split3 && splith && !(o.dbg & 8);
            // heads as the A operand of two 32x32x16 steps: [plane][step], row = head (lane & 31;
            // rows >= 6 zero), k-slot (s, hk, i) = channel 16 s + 8 (i >> 2) + (i & 3) + 4 hk --
            // exactly the conv3 accumulator registers 8 s + i of lane half hk (mtcnn_runtime packs
            // [2][32][32] halves that way)
            f16x8 hw[2][2] = {};
            if (c3_32) {
                int ln = lane;
                asm volatile("" : "+v"(ln));
                const int hoff = ((ln & 31) * 32 + 8 * (ln >> 5)) * 2;
#pragma unroll
                for (int pl = 0; pl < 2; pl++)
#pragma unroll
                    for (int s = 0; s < 2; s++)
                        hw[pl][s] = __builtin_bit_cast(
                            f16x8, __builtin_amdgcn_raw_buffer_load_b128(rhh, hoff, pl * 32 * 32 * 2 + s * 32, 0));
            }
            // (issued after the head weights: loads complete in order, and the frame bytes are
            //  the slow ones; the scheduling barrier keeps the order)
            __builtin_amdgcn_sched_barrier(0);
            {
                // the loads are issued on every tile (a dummy read of the first frame byte when
                // there is nothing to prefetch), so both paths leave the same count of loads in
                // flight and the waits for the head weights above stay partial
                const uint8_t* pf_src = frames;
                int qw3 = 1, nb2 = 1, pf_rows = 0;
                const int64_t nt = __builtin_amdgcn_readfirstlane(s_next);
                if (nt < total_tiles && !(o.dbg & 64)) {
                    int L2 = L;  // nt > blk
                    while (L2 + 1 < n_levels && nt >= lvc[L2 + 1].tile_beg) L2++;
                    const PNetLevel Q = load_level(lvc + L2);
                    if (!Q.pre) {
                        const TileGeo g2 = tile_geo<VR>((int)(nt - Q.tile_beg), Q);
                        const int b2i = g2.b;
                        const int oy2 = g2.ty * PT_H, ox2 = g2.tx * PT_W;
                        // (the next tile's first level row: VR_LROW when it continues this one)
                        const int lr2 = VR && nt == blk + 1 && g2.ty > 0 ? VR_LROW : 0;
                        const int ry = min(PL_H - 1, Q.lh - 1 - 2 * oy2), rx = min(PL_W - 1, Q.lw - 1 - 2 * ox2);
                        const int gy0 = udiv_est((2 * oy2 + lr2) * H, Q.lh), gy1 = udiv_est((2 * oy2 + ry + 1) * H + Q.lh - 1, Q.lh);
                        const int gx0 = udiv_est(2 * ox2 * W, Q.lw), gx1 = udiv_est((2 * ox2 + rx + 1) * W + Q.lw - 1, Q.lw);
                        const int w3 = (gx1 - gx0) * 3, nb = (gy1 - gy0) * w3;
                        if ((int64_t)(gy1 - gy0) * w3 <= LP::PATCH && nb > 0) {
                            pf_src = frames + (int64_t)b2i * frame_stride + (int64_t)gy0 * row_stride + gx0 * 3;
                            qw3 = w3;
                            nb2 = nb;
                            pf_rows = 1;
                        }
                    }
                }
                const int ext = pf_rows ? (nb2 / qw3 - 1) * (int)row_stride + qw3 : 1;
                pfv = patch_bytes8(__builtin_amdgcn_make_buffer_rsrc((void*)pf_src, 0, ext, 0x00020000), 8 * tid, qw3,
                                   (int)row_stride);
                pf_n = pf_rows ? nb2 : 0;
            }
            // head biases of the lane's accumulator rows 4 lkx + i (group 0: conv4_1 0, 1, conv4_2
            // 0, 1; group 1: conv4_2 2, 3; groups 2, 3 hold no heads)
            const f32x4 hbv = lkx == 0 ? f32x4{wf[PW_C41B], wf[PW_C41B + 1], wf[PW_C42B], wf[PW_C42B + 1]}
                                       : f32x4{wf[PW_C42B + 2], wf[PW_C42B + 3], 0.f, 0.f};
            // stage-1 gate of one cell: softmax over the face logits (mtcnn.py:37), p >= 0.6
            // (mtcnn.py:183), wave-aggregated candidate append; DENSE writes the parity maps
            auto gate = [&](bool valid, int oy, int ox, float a0, float a1v, float q0, float q1, float q2, float q3) {
                auto softmax1 = [&]() {
                    const float mx = fmaxf(a0, a1v);
                    const float e0 = expf(a0 - mx), e1 = expf(a1v - mx);
                    return __fdiv_rn(e1, e0 + e1);
                };
                if (DENSE) {
                    const float prob = softmax1();
                    if (valid) {
                        int64_t plane = (int64_t)P.ph * P.pw;
                        int64_t pc = (int64_t)oy * P.pw + ox;
                        o.prob[(int64_t)b * plane + pc] = prob;
                        float* rg = o.reg + (int64_t)b * 4 * plane + pc;
                        rg[0] = q0;
                        rg[plane] = q1;
                        rg[2 * plane] = q2;
                        rg[3 * plane] = q3;
                    }
                } else {
                    // mask = prob >= 0.6 (the python scalar compares as fp32).  The softmax is
                    // evaluated only where it can pass: with d = a1 - a0 (the same fp32 difference
                    // the reference exponentiates when a1 > a0), d < 0.4 gives prob <= 1 / (1 +
                    // expf(-0.4)) = 0.5987 < 0.6, a margin far above expf's and the division's
                    // rounding; a NaN d takes the exact path.  ~0.1 % of the cells pass, so nearly
                    // every wave skips the two expf and the division (wave-uniform branch).
                    const bool near = valid && !(a1v - a0 < 0.4f) && !(o.dbg & 16);
                    float prob = 0.f;
                    bool pass = false;
                    if (__ballot(near)) {
                        prob = softmax1();
                        pass = near && prob >= 0.6f;
                    }
                    uint64_t bal = __ballot(pass);
                    if (bal) {
                        int leader = __builtin_ctzll(bal);
                        uint32_t base = 0;
                        if (lane == leader) {
                            base = atomicAdd(o.count, (uint32_t)__popcll(bal));
                            atomicAdd(&o.level_count[L], (uint32_t)__popcll(bal));
                        }
                        base = __shfl(base, leader);
                        if (pass) {
                            uint32_t slot = base + (uint32_t)__popcll(bal & ((1ull << lane) - 1ull));
                            if (slot < o.cap) {
                                uint32_t lin = (uint32_t)(((int64_t)b * P.ph + oy) * P.pw + ox);
                                o.key[slot] = ((uint64_t)L << 32) | lin;
                                o.score[slot] = prob;
                                o.regv[slot] = make_float4(q0, q1, q2, q3);
                            }
                        }
                    }
                }
            };
            if (c3_32) {
                // conv3 (16 -> 32, 3x3) transposed on v_mfma_f32_32x32x16_f16: C (32 channels x 32
                // cells) = W3 (32 x 144) x im2col (144 x 32 cells), one k-step per tap (16 channels,
                // K = 144 exactly: no padding slots).  A = the split weights in LDS (row = channel
                // lane & 31, k = 16 tap + 8 hk ..), B = conv2's split output (column = cell lane & 31).
                // Main products x0 w0 into an accumulator seeded with the bias, the cross terms x0 w1 +
                // x1 w0 into a second one; 27 MFMAs per 32 cells (60 of 16x16x32 before, 8 issue
                // cycles each).  Accumulator register r of lane l: channel (r & 3) + 8 (r >> 2) + 4 hk
                // of cell l & 31; both heads are two more 32x32x16 steps over those registers.
                typedef __attribute__((ext_vector_type(16))) float f32x16;
                typedef const volatile __attribute__((address_space(3))) f32x4 lds_f32x4;
                constexpr int NPOS = PC_H * PC_W;
                const _Float16* sH = (const _Float16*)sA;
                int ln = lane;
                asm volatile("" : "+v"(ln));
                const int c32 = ln & 31, hk = ln >> 5;
                // (rows >= 16 hold each tap's channel halves swapped, see C3_SWZ)
                const _Float16* sWh = (const _Float16*)(sP + LP::W3) + c32 * W3_ROW + 8 * (hk ^ (c32 >> 4));
                const float* cst = s_c3 + 16 * hk;  // [bias | slope] rows of the lane half
                const f32x4 hb = hk == 0 ? f32x4{wf[PW_C41B], wf[PW_C41B + 1], wf[PW_C42B], wf[PW_C42B + 1]}
                                         : f32x4{wf[PW_C42B + 2], wf[PW_C42B + 3], 0.f, 0.f};
#pragma unroll 1
                for (int hh = 0; hh < NHALF; hh++) {
                    const int cell = (wave * FPW + hh * FH) * 16 + c32;
                    const int cy = cell / PT_W, cx = cell % PT_W;
                    // (cy = even first row + c32 >> 4; odd conv2 rows swapped: the half this lane reads
                    //  flips with the tap row's parity)
                    const _Float16* xs = sH + (cy * PC_W + cx) * 16 + 8 * (hk ^ (c32 >> 4));
                    const _Float16* xsf = sH + (cy * PC_W + cx) * 16 + 8 * (hk ^ (c32 >> 4) ^ 1);
                    f32x16 am, ac = {};
#pragma unroll
                    for (int i = 0; i < 4; i++) {
                        const f32x4 v = *(lds_f32x4*)(cst + 4 * i);
                        am[4 * i] = v[0], am[4 * i + 1] = v[1], am[4 * i + 2] = v[2], am[4 * i + 3] = v[3];
                    }
                    // operands one tap ahead (two register stages; the scheduling barriers keep
                    // the compiler from hoisting all 36 reads, which would spill)
                    f16x8 op[2][4];
                    auto ld_tap = [&](int t, f16x8* d) {
                        const int to = ((t / 3) * PC_W + t % 3) * 16;
                        d[0] = *(const f16x8*)(sWh + 16 * t);
                        d[1] = *(const f16x8*)(sWh + 32 * W3_ROW + 16 * t);
                        const _Float16* xt = ((t / 3) & 1) ? xsf : xs;
                        d[2] = *(const f16x8*)(xt + to);
                        d[3] = *(const f16x8*)(xt + NPOS * 16 + to);
                    };
                    ld_tap(0, op[0]);
#pragma unroll
                    for (int t = 0; t < 9; t++) {
                        if (t + 1 < 9) ld_tap(t + 1, op[(t + 1) & 1]);
                        const f16x8* c = op[t & 1];
                        am = __builtin_amdgcn_mfma_f32_32x32x16_f16(c[0], c[2], am, 0, 0, 0);
                        ac = __builtin_amdgcn_mfma_f32_32x32x16_f16(c[1], c[2], ac, 0, 0, 0);
                        ac = __builtin_amdgcn_mfma_f32_32x32x16_f16(c[0], c[3], ac, 0, 0, 0);
                        __builtin_amdgcn_sched_barrier(0);
                    }
                    if (o.dbg & 32) continue;
                    auto epi = [&](auto u_t) {
                        constexpr bool U3 = decltype(u_t)::value;
                        // 2048 (bias + main) + cross, PReLU (commutes with the scaling), split
                        f16x8 x0h[2], x1h[2];
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            const f32x4 a = *(lds_f32x4*)(cst + 32 + 4 * i);
#pragma unroll
                            for (int k = 0; k < 4; k++) {
                                const int r = 4 * i + k;
                                _Float16 p0, p1;
                                split_u(prelu_t<U3>(fmaf(am[r], 2048.f, ac[r]), a[k]), p0, p1);
                                x0h[r >> 3][r & 7] = p0;
                                x1h[r >> 3][r & 7] = p1;
                            }
                        }
                        // heads: cross terms first, scaled by 2^-11 into the main products' chain
                        f32x16 hc = {};
#pragma unroll
                        for (int s = 0; s < 2; s++) {
                            hc = __builtin_amdgcn_mfma_f32_32x32x16_f16(hw[0][s], x1h[s], hc, 0, 0, 0);
                            hc = __builtin_amdgcn_mfma_f32_32x32x16_f16(hw[1][s], x0h[s], hc, 0, 0, 0);
                        }
                        // (only registers 0..3 hold head rows -- 0..3 in lane half 0, 4, 5 in half 1;
                        //  the rest are the zero rows >= 8 -- so only they are scaled)
#pragma unroll
                        for (int r = 0; r < 4; r++) hc[r] = hc[r] * 0.00048828125f;
#pragma unroll
                        for (int s = 0; s < 2; s++)
                            hc = __builtin_amdgcn_mfma_f32_32x32x16_f16(hw[0][s], x0h[s], hc, 0, 0, 0);
                        // registers 0..3 of lane half 0: heads 0..3 (a0 a1 r0 r1), of half 1: heads
                        // 4, 5 (r2 r3); biases added (VALU) before the swap that hands half 1's r2,
                        // r3 to half 0 (lanes l and l + 32 hold the same cell)
                        const f32x4 hq = f32x4{hc[0], hc[1], hc[2], hc[3]} + hb;
                        const auto s2 = __builtin_amdgcn_permlane32_swap(__float_as_uint(hq[0]), __float_as_uint(hq[0]), false, false);
                        const auto s3 = __builtin_amdgcn_permlane32_swap(__float_as_uint(hq[1]), __float_as_uint(hq[1]), false, false);
                        const int oy = oy0 + cy, ox = ox0 + cx;
                        const bool valid = hk == 0 && oy < P.ph && ox < P.pw;
                        gate(valid, oy, ox, hq[0], hq[1], hq[2], hq[3], __uint_as_float(s2[1]), __uint_as_float(s3[1]));
                    };
                    if (wg.unit_slopes & 2)
                        epi(std::true_type{});
                    else
                        epi(std::false_type{});
                }
            } else
#pragma unroll 1
            for (int hh = 0; hh < NHALF; hh++) {
                f32x4 acc[FH][2];
    #pragma unroll
                for (int j = 0; j < FH; j++) acc[j][0] = acc[j][1] = f32x4{0.f, 0.f, 0.f, 0.f};
                int ab[FH];
    #pragma unroll
                for (int j = 0; j < FH; j++) {
                    const int cell = (wave * FPW + hh * FH + j) * 16 + lrx;
                    ab[j] = (cell / PT_W) * PC_W + (cell % PT_W);
                }
                const int nchunk = (o.dbg & 8) || split3 ? 0 : 4;
                if (split3 && !(o.dbg & 8)) {
                    // fp16 matrix cores, K = 9 taps x 16 ch in 5 steps of 32 (tap 9 = zero weights):
                    // lane group lkx holds 8 channels (8 * (lkx & 1) ...) of tap 2s + (lkx >> 1), one
                    // 16-byte LDS read per part; main products x0 w0 and the 2^11-scaled cross terms
                    // x0 w1 + x1 w0 go to separate accumulators, combined once at the end
                    constexpr int NPOS = PC_H * PC_W;
                    const _Float16* sH = (const _Float16*)sA;
                    f32x4 accc[FH][2];
    #pragma unroll
                    for (int j = 0; j < FH; j++) accc[j][0] = accc[j][1] = f32x4{0.f, 0.f, 0.f, 0.f};
                    // weights from the pooled buffer (rows of W3_ROW halves); k slots >= 144 (step 4,
                    // lane groups 2, 3) are zero: those lanes read the zero pad after the level planes
                    const _Float16* sWh = (const _Float16*)(sP + LP::W3) + lrx * W3_ROW + 8 * lkx;
                    const _Float16* sWhs = (const _Float16*)(sP + LP::W3) + lrx * W3_ROW + 8 * (lkx ^ 1);  // rows >= 16
                    const _Float16* zpad = (const _Float16*)(sA + LP::A - 4);
    #pragma unroll
                    for (int s5 = 0; s5 < 5; s5++) {
                        f16x8 w0[2], w1[2];
                        const bool zw = s5 == 4 && lkx >= 2;
    #pragma unroll
                        for (int mf = 0; mf < 2; mf++) {
                            const _Float16* sw = mf ? sWhs : sWh;
                            w0[mf] = *(const f16x8*)(zw ? zpad : sw + (mf * 16) * W3_ROW + 32 * s5);
                            w1[mf] = *(const f16x8*)(zw ? zpad : sw + (32 + mf * 16) * W3_ROW + 32 * s5);
                        }
                        const int tap = min(2 * s5 + (lkx >> 1), 8);
                        const int xo = ((tap / 3) * PC_W + (tap % 3)) * 16;
                        const int hx = 8 * ((lkx & 1) ^ ((tap / 3) & 1));  // + the cell row's parity (j & 1)
    #pragma unroll
                        for (int j = 0; j < FH; j++) {
                            const int xj = xo + (hx ^ (8 * (j & 1)));
                            const f16x8 x0 = *(const f16x8*)(sH + ab[j] * 16 + xj);
                            const f16x8 x1 = *(const f16x8*)(sH + NPOS * 16 + ab[j] * 16 + xj);
    #pragma unroll
                            for (int mf = 0; mf < 2; mf++) {
                                acc[j][mf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0[mf], x0, acc[j][mf], 0, 0, 0);
                                accc[j][mf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w1[mf], x0, accc[j][mf], 0, 0, 0);
                                accc[j][mf] = __builtin_amdgcn_mfma_f32_16x16x32_f16(w0[mf], x1, accc[j][mf], 0, 0, 0);
                            }
                        }
                    }
    #pragma unroll
                    for (int j = 0; j < FH; j++)
    #pragma unroll
                        for (int mf = 0; mf < 2; mf++)
    #pragma unroll
                            for (int i = 0; i < 4; i++) acc[j][mf][i] = fmaf(acc[j][mf][i], 2048.f, accc[j][mf][i]);
                }
                // k-step s = (tap s/4, channel 4*(s%4) + lkx): the LDS offset is the lane-group base
                // lkx * plane plus a compile-time constant (an instruction immediate, no registers)
                const float* sAl = sA + lkx * (PC_H * PC_W);
                const int w3off = (lkx * 9 * 32 + lrx) * 4;
    #pragma unroll
                for (int sc = 0; sc < 4; sc++) {
                    if (sc >= nchunk) break;
                    float w3[9][2];
    #pragma unroll
                    for (int t = 0; t < 9; t++) {
                        const int st = 9 * sc + t, tap = st >> 2, cq = st & 3;
                        w3[t][0] = __uint_as_float(__builtin_amdgcn_raw_buffer_load_b32(rw3, w3off, ((4 * cq * 9 + tap) * 32) * 4, 0));
                        w3[t][1] = __uint_as_float(
                            __builtin_amdgcn_raw_buffer_load_b32(rw3, w3off, ((4 * cq * 9 + tap) * 32 + 16) * 4, 0));
                    }
    #pragma unroll
                    for (int t = 0; t < 9; t++) {
                        const int st = 9 * sc + t, tap = st >> 2, cq = st & 3;
                        const int ko = 4 * cq * PC_H * PC_W + (tap / 3) * PC_W + (tap % 3);
    #pragma unroll
                        for (int j = 0; j < FH; j++) {
                            const float bv = sAl[ab[j] + ko];
                            acc[j][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(w3[t][0], bv, acc[j][0], 0, 0, 0);
                            acc[j][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w3[t][1], bv, acc[j][1], 0, 0, 0);
                        }
                    }
                }
                if (nchunk > 0) {  // fp32 path: accumulators to the 2048-scaled form (exact)
    #pragma unroll
                    for (int j = 0; j < FH; j++) acc[j][0] *= 2048.f, acc[j][1] *= 2048.f;
                }
                static_assert(FH == 2, "the heads epilogue pairs the two fragments of a pass");
                // conv3 epilogue + both 1x1 heads per fragment, then the pair's head values
                // regrouped so one softmax / gate per lane covers both fragments (U3: conv3's
                // PReLU slope class)
                auto heads = [&](auto u_t) {
                    constexpr bool U3 = decltype(u_t)::value;
                    f32x4 hq[FH];
    #pragma unroll
                    for (int j = 0; j < FH; j++) {
                        f32x4 hacc = {0.f, 0.f, 0.f, 0.f};
                        // (the split heads run on the 32x32 path above: here the fp32 heads)
    #pragma unroll
                        for (int i = 0; i < 4; i++) {
                            const float fa = prelu_t<U3>(acc[j][0][i] + cb3[0][i], ca3[0][i]) * 0.00048828125f;
                            const float fb = prelu_t<U3>(acc[j][1][i] + cb3[1][i], ca3[1][i]) * 0.00048828125f;
                            hacc = __builtin_amdgcn_mfma_f32_16x16x4f32(hwA[0][i], fa, hacc, 0, 0, 0);
                            hacc = __builtin_amdgcn_mfma_f32_16x16x4f32(hwA[1][i], fb, hacc, 0, 0, 0);
                        }
                        // head biases added here, per lane group (group 0: a0 a1 r0 r1, group 1: r2
                        // r3): the swap below then reads a VALU result -- the compiler's wait-state
                        // count for v_permlane16_swap reading a 16x16x4 f32 MFMA result directly is
                        // two short of the one it gives other VALU reads (stale values, seen on the
                        // fp32 path)
                        hq[j] = hacc + hbv;
                    }
                    // hq[j]: lane (cell lrx, heads 4 lkx + i): group 0 = (a0, a1, r0, r1), group 1 =
                    // (r2, r3, -, -).  One permlane16_swap per register moves fragment 1's group-0
                    // values into group 1 of hq[0] and fragment 0's group-1 values into group 0 of
                    // hq[1]: lane groups 0 / 1 then hold fragment 0 / 1 whole, in the same registers
    #pragma unroll
                    for (int k = 0; k < 4; k++) {
                        const auto sw = __builtin_amdgcn_permlane16_swap(__float_as_uint(hq[0][k]), __float_as_uint(hq[1][k]), false, false);
                        hq[0][k] = __uint_as_float(sw[0]);
                        hq[1][k] = __uint_as_float(sw[1]);
                    }
                    const int cell = (wave * FPW + hh * FH + (lkx & 1)) * 16 + lrx;
                    const int y = cell / PT_W, x = cell % PT_W;
                    const int oy = oy0 + y, ox = ox0 + x;
                    const bool valid = (lkx < 2) && (oy < P.ph) && (ox < P.pw);
                    gate(valid, oy, ox, hq[0][0], hq[0][1], hq[0][2], hq[0][3], hq[1][0], hq[1][1]);
                };
                if (!(o.dbg & 32)) {
                    if (wg.unit_slopes & 2)
                        heads(std::true_type{});
                    else
                        heads(std::false_type{});
                }
            }
        }
        if (X || (PR && pf_n > 0)) __syncthreads();  // conv3's weights (under the patch bytes) are no longer read
        if (pf_n > 0 && 8 * tid < pf_n) *(uint2*)((uint8_t*)sP + 8 * tid) = pfv;
        pf_done = pf_n > 0;
        if (tid == 0) {  // every thread read s_tile / s_cend before this tile's barriers
            s_tile = (int)next_tile;
            s_cend = (int)next_cend;
        }
        __syncthreads();  // sA/sP are rewritten by the next tile
        mark(6);  // 6: prefetch issue, conv3, heads, gate
    }
    if (clk_on && tid < 8) atomicAdd(&o.clk[tid], s_clk[tid]);
}

// tiles of the leading levels the exact-levels variant can take: upsampled (lh >= H, lw >= W,
// no precomputed level) and every tile's frame patch + 8-byte row sums within its staging buffer
// (bounds: a tile's 42-pixel level span covers at most 42 H / lh + 2 frame rows / columns)
int64_t pnet_pre_from(const std::vector<PNetLevel>& lv, int64_t total_tiles) {
    int64_t from = total_tiles;
    for (size_t i = lv.size(); i-- > 0;) {
        if (!(lv[i].pre && lv[i].pad == 1)) break;
        from = lv[i].tile_beg;
    }
    return from;
}

int64_t pnet_exact_tiles(const std::vector<PNetLevel>& lv, int H, int W, int64_t total_tiles) {
    for (const auto& L : lv) {
        const int rows = (PL_H * H + L.lh - 1) / L.lh + 2, cols = (PL_W * W + L.lw - 1) / L.lw + 2;
        const int hs_off = (rows * cols * 3 + 7) & ~7;
        const bool fits = rows * cols * 3 <= PnLds<true>::PATCH && hs_off + rows * PL_W * 8 <= PnLds<true>::PATCH;
        if (L.lh < H || L.lw < W || L.pre || !fits || W >= 128 * L.lw) return L.tile_beg;
    }
    return total_tiles;
}

static_assert(PNET_VR_SLOT == VR_SLOT, "mtcnn.hpp's VR slot size");

// tiles per atomic chunk (VTF_PNET_CHUNK) and chunks per workgroup (VTF_PNET_QUOTA, 0 = persistent)
static void pnet_chunking(int& chunk, int& quota) {
    // (clamped: the kernel keeps tile indices and chunk ends in int)
    const char* ce = std::getenv("VTF_PNET_CHUNK");
    chunk = ce && std::atoi(ce) > 0 ? std::min(64, std::atoi(ce)) : PNET_TILE_CHUNK;
    // (chunk x quota at 8 tiles per workgroup, full default run: 4 x 2 12.26-12.30k, 2 x 4
    // 12.19-12.21k, 1 x 8 12.18k faces/s; round 6, distinct frames and the 2 ms lane stagger:
    // 4 x 1 10.00-10.03k against 4 x 2 9.91-9.97k, 4 x 4 9.80-9.85k, and the pair solo 4.229 vs
    // 4.282 ms -- profiles/r06_pnet_quota_ab.txt)
    const char* qe = std::getenv("VTF_PNET_QUOTA");
    quota = qe ? std::min(1 << 16, std::max(0, std::atoi(qe))) : 1;
}

static int pnet_cus() {
    int dev = 0, cus = 256;
    VTF_HIP(hipGetDevice(&dev));
    VTF_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    return cus;
}

static int pnet_wgs(const char* name, int mx) {
    const char* e = std::getenv(name);
    const int v = e ? std::atoi(e) : 0;
    return v >= 1 && v <= mx ? v : mx;
}

// grid of the exact-levels launch over `exact_tiles` tiles (the vertical-reuse slots it needs)
int64_t pnet_x_grid(int64_t exact_tiles) {
    if (exact_tiles <= 0) return 0;
    int chunk = 0, quota = 0;
    pnet_chunking(chunk, quota);
    int64_t grid = std::min<int64_t>(exact_tiles, (int64_t)pnet_cus() * pnet_wgs("VTF_PNET_X_WG_PER_CU", PnLds<true>::GPC));
    if (quota > 0) grid = std::max<int64_t>(grid, (exact_tiles + (int64_t)quota * chunk - 1) / ((int64_t)quota * chunk));
    return grid;
}

void launch_pnet(bool dense, const uint8_t* frames, int64_t frame_stride, int64_t row_stride, int H, int W,
                 const PNetLevel* d_levels, int n_levels, int64_t total_tiles, const PNetW& w, const PNetOut& o,
                 uint32_t* d_tile_ctr, hipStream_t st, int64_t exact_tiles, int64_t pre_from) {
    if (total_tiles <= 0) return;
    VTF_CHECK(H < 65536 && W < 65536, VTF_E_LIMIT, "mtcnn: frames must be smaller than 65536 px per side");
    // k_pnet's index math is 32-bit (udiv_est): tile indices and bin numerators below 2^31
    VTF_CHECK(total_tiles < (int64_t)1 << 30, VTF_E_LIMIT, "mtcnn: too many PNet tiles in one launch");
    // frame patches are read through 32-bit buffer offsets (patch_bytes8)
    VTF_CHECK(row_stride > 0 && row_stride < (int64_t)1 << 24, VTF_E_LIMIT, "mtcnn: frame row stride too large");
    // (level sizes: checked where the level plan is built, mtcnn_runtime)
    const int cus = pnet_cus();
    // persistent workgroups per CU: the variant's LDS limit fills every CU; a smaller count leaves
    // room for concurrently running lanes' kernels (env VTF_PNET_WG_PER_CU / VTF_PNET_X_WG_PER_CU,
    // experiments).  Tiles [0, exact_tiles) -- the leading upsampled levels, checked on the host --
    // run on the exact-levels variant (X, four workgroups per CU) when the split mode is on
    // (VTF_PNET_X=0: one launch of the general kernel).
    auto wgs = pnet_wgs;
    const char* xe = std::getenv("VTF_PNET_X");
    // chunks per workgroup (VTF_PNET_QUOTA, 0 = persistent: every workgroup runs to the end of the
    // tile range): with a quota the grid is ~tiles / (quota * chunk) workgroups that retire as they
    // finish, so other lanes' kernels get CU slots during the launch instead of after it (a
    // persistent launch holds every CU's registers and LDS for its whole ~4.5 ms).  c2 3 lanes:
    // persistent 11.60-11.80k, quota 16 / 8 / 4 / 2: 11.98-11.99k / 12.20-12.23k / 12.34-12.39k /
    // 12.31-12.37k faces/s (same box)
    int chunk = 0, quota = 0;
    pnet_chunking(chunk, quota);
    if (!w.c3h || !w.hh || dense || (xe && std::atoi(xe) == 0)) exact_tiles = 0;
    exact_tiles = std::min(exact_tiles, total_tiles);
    // (d_tile_ctr: three counters the caller zeroed, one per launch -- no fill kernels here)
    if (exact_tiles > 0) {
        const int64_t grid = pnet_x_grid(exact_tiles);
        // vertical reuse (VTF_PNET_VR=1: on) when the caller provided a slot per workgroup
        const char* ve = std::getenv("VTF_PNET_VR");
        if (o.vr && grid <= o.vr_slots && ve && std::atoi(ve) != 0)
            k_pnet<false, true, false, true><<<(unsigned)grid, 256, 0, st>>>(
                frames, frame_stride, row_stride, H, W, d_levels, n_levels, exact_tiles, d_tile_ctr, w, o, 0, quota, chunk);
        else
            k_pnet<false, true><<<(unsigned)grid, 256, 0, st>>>(frames, frame_stride, row_stride, H, W, d_levels, n_levels,
                                                                 exact_tiles, d_tile_ctr, w, o, 0, quota, chunk);
    }
    if (exact_tiles >= total_tiles) return;
    // the trailing levels precomputed as split pixels run on the PR variant (four workgroups per CU)
    // when the split mode is on (VTF_PNET_PR=0: the general kernel takes them)
    const char* pe = std::getenv("VTF_PNET_PR");
    if (!w.c3h || !w.hh || dense || (pe && std::atoi(pe) == 0)) pre_from = total_tiles;
    pre_from = std::max(exact_tiles, std::min(pre_from, total_tiles));
    PNetOut og = o;  // (phase clocks of the launches after X in words 8..15)
    if (og.clk && exact_tiles > 0) og.clk += 8;
    if (pre_from > exact_tiles) {  // general variant: tiles [exact_tiles, pre_from)
        const int64_t rest = pre_from - exact_tiles;
        int64_t grid = std::min<int64_t>(rest, (int64_t)cus * wgs("VTF_PNET_WG_PER_CU", PnLds<false>::GPC));
        if (quota > 0) grid = std::max<int64_t>(grid, (rest + (int64_t)quota * chunk - 1) / ((int64_t)quota * chunk));
        if (dense)
            k_pnet<true, false><<<(unsigned)grid, 256, 0, st>>>(frames, frame_stride, row_stride, H, W, d_levels, n_levels,
                                                                 pre_from, d_tile_ctr + 1, w, og, exact_tiles, quota, chunk);
        else
            k_pnet<false, false><<<(unsigned)grid, 256, 0, st>>>(frames, frame_stride, row_stride, H, W, d_levels, n_levels,
                                                                  pre_from, d_tile_ctr + 1, w, og, exact_tiles, quota, chunk);
    }
    if (pre_from < total_tiles) {  // PR variant: tiles [pre_from, total_tiles)
        const int64_t rest = total_tiles - pre_from;
        int64_t grid = std::min<int64_t>(rest, (int64_t)cus * PnLds<true>::GPC);
        if (quota > 0) grid = std::max<int64_t>(grid, (rest + (int64_t)quota * chunk - 1) / ((int64_t)quota * chunk));
        const char* ve = std::getenv("VTF_PNET_VR");
        if (o.vr && grid <= o.vr_slots && ve && std::atoi(ve) != 0)
            k_pnet<false, false, true, true><<<(unsigned)grid, 256, 0, st>>>(
                frames, frame_stride, row_stride, H, W, d_levels, n_levels, total_tiles, d_tile_ctr + 2, w, og, pre_from,
                quota, chunk);
        else
            k_pnet<false, false, true><<<(unsigned)grid, 256, 0, st>>>(frames, frame_stride, row_stride, H, W, d_levels,
                                                                        n_levels, total_tiles, d_tile_ctr + 2, w, og,
                                                                        pre_from, quota, chunk);
    }
}

// ----------------------------------------------------------------------------------- RNet / ONet
// The candidate networks run as batched layers on the MFMA implicit-GEMM conv kernel
// (conv.hip, fp32, PReLU epilogue); here: the crop front end and the tiny heads.

// Fused candidate front end: _get_cropped_candidates (mtcnn.py:153-163) + conv1 (3->28/32,
// 3x3) + PReLU + MaxPool2d(3, 2, ceil_mode) of RNet (S=24) / ONet (S=48), one candidate per
// workgroup.  The S x S crop is adaptive-pooled from the uint8 frame straight into LDS
// (bit-exact bins), conv1 runs on fp32 MFMA with the true K = 27 (im2col order (c, ky, kx),
// no channel padding), and the pool reads the conv1 band from LDS: only the pooled
// [n, P, P, 32] map reaches HBM (P = 11 / 23).  Conv rows are produced 2*PB per band into a
// ring of 2*PB+1 rows (the pool window's shared row is kept, not recomputed).
// w1: [28][32] (k, co; row 27 and channels >= Cout zero); b1, a1: [32].
template <int S, int PB, int NT, bool XS>
__global__ __launch_bounds__(NT) void k_cand_front(const void* __restrict__ sat, int pk, int H, int W,
                                                   const float4* __restrict__ boxes, const int32_t* __restrict__ img,
                                                   const float* __restrict__ w1, const _Float16* __restrict__ w1h,
                                                   const float* __restrict__ b1, const float* __restrict__ a1,
                                                   float* __restrict__ out, int32_t* __restrict__ err, int dbg,
                                                   int* __restrict__ ovf) {
    constexpr int O = S - 2;                // conv1 output side
    constexpr int P = (O - 3 + 1) / 2 + 1;  // ceil-mode pool output side
    constexpr int BR = 2 * PB + 1;          // conv rows per band
    constexpr int NW = NT / 64;
    constexpr int PIX = (S * S + NT - 1) / NT;  // crop pixels per thread
    // conv ring [32 ch][CS]: an odd channel stride puts the 32 channels a pool read spans on
    // 32 distinct banks
    constexpr int CS = (BR * O) | 1;
    // crop: fp32 channel planes [3][S*S], or (XS) fp16 split planes [2][S*S + 1][4] (R, G, B, 0;
    // one zero pixel after each plane: the conv operand reads run one pixel past the last one,
    // against zero weights)
    constexpr int CROP_F = XS ? 4 * (S * S + 1) : 3 * S * S;
    __shared__ __attribute__((aligned(16))) float crop[CROP_F];
    __shared__ float cv[32 * CS];
    const int64_t k = blockIdx.x;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lk = lane >> 4;
    float* o = out + k * (P * P * 32);
    int y0, x0, hc, wc;
    if (!crop_rect(boxes[k], H, W, y0, x0, hc, wc)) {
        // the reference skips this box and then fails indexing (IndexError): flag it
        if (tid == 0) atomicAdd(err, 1);
        for (int i = tid; i < P * P * 32; i += NT) o[i] = 0.f;
        return;
    }
    // upsampled crops (box within S x S): bins of 1 or 2 pixels per side, every value s / 2^(8..10)
    // with |s| <= 1020 -- exact in fp16, so the residual plane is zero and skipped
    const bool exact = XS && hc <= S && wc <= S;
    typedef __attribute__((ext_vector_type(4))) _Float16 h4;
    h4* cp0 = (h4*)crop;
    h4* cp1 = cp0 + (S * S + 1);
    if (XS && tid == 0) {
        const h4 z = {(_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
        cp0[S * S] = z;
        cp1[S * S] = z;
    }
    // crop bins from the SAT: every thread issues all of its corner loads before using any
    // (the gathers are latency-bound; PIX * 4 loads in flight per thread)
    const int64_t sk = (int64_t)img[k] * (H + 1) * (W + 1);
    if (!(dbg & 1)) {
        int idx[PIX], kh[PIX], kw[PIX];
        int3 sm[PIX];
#pragma unroll
        for (int j = 0; j < PIX; j++) idx[j] = min(tid + j * NT, S * S - 1);
        if (pk)
            crop_bins<PIX, S, true>(sat, sk, W + 1, y0, x0, hc, wc, idx, sm, kh, kw);
        else
            crop_bins<PIX, S, false>(sat, sk, W + 1, y0, x0, hc, wc, idx, sm, kh, kw);
#pragma unroll
        for (int j = 0; j < PIX; j++) {
            const int i = tid + j * NT;
            if (i < S * S) {
                const float r = bin_avg(sm[j].x, kh[j], kw[j]);
                const float g = bin_avg(sm[j].y, kh[j], kw[j]);
                const float bl = bin_avg(sm[j].z, kh[j], kw[j]);
                if (XS) {
                    _Float16 r0, r1, g0, g1, b0, b1_;
                    split_f16(r, r0, r1);
                    split_f16(g, g0, g1);
                    split_f16(bl, b0, b1_);
                    cp0[i] = h4{r0, g0, b0, (_Float16)0.f};
                    if (!exact) cp1[i] = h4{r1, g1, b1_, (_Float16)0.f};
                } else {
                    crop[i] = r;
                    crop[S * S + i] = g;
                    crop[2 * S * S + i] = bl;
                }
            }
        }
    }
    // conv1 weights: fp32 [28][32] (k, co) for the fp32 MFMA path, or the split planes [2][32][64]
    // (k = ky*16 + kx*4 + c) as the B operand of 16x16x32 fp16 MFMAs, channel block nb = co / 16
    float wb[XS ? 1 : 7][2];
    f16x8 wh0[XS ? 2 : 1][2], wh1[XS ? 2 : 1][2];
    if (XS) {
#pragma unroll
        for (int s2 = 0; s2 < 2; s2++)
#pragma unroll
            for (int nb = 0; nb < 2; nb++) {
                const _Float16* src = w1h + (16 * nb + lr) * 64 + 32 * s2 + 8 * lk;
                wh0[s2][nb] = *(const f16x8*)src;
                wh1[s2][nb] = *(const f16x8*)(src + 32 * 64);
            }
    } else {
#pragma unroll
        for (int s = 0; s < 7; s++) {
            wb[s][0] = w1[(4 * s + lk) * 32 + lr];
            wb[s][1] = w1[(4 * s + lk) * 32 + 16 + lr];
        }
    }
    const float bb0 = b1[lr], bb1 = b1[16 + lr], aa0 = a1[lr], aa1 = a1[16 + lr];
    __syncthreads();
    // conv rows live in a ring of BR rows (slot = row % BR): a band's first row (2*pr0) is the
    // previous band's last, so each band computes only its 2*PB new rows
    for (int pr0 = 0; pr0 < P; pr0 += PB) {
        const int cr0 = 2 * pr0;
        const int r_lo = pr0 == 0 ? 0 : cr0 + 1;
        const int r_hi = min(cr0 + 2 * PB, O - 1);
        const int npos = (r_hi - r_lo + 1) * O;
        const int nf = npos > 0 && !(dbg & 2) ? (npos + 15) / 16 : 0;
        for (int f = wave; f < nf; f += NW) {
            const int p = min(f * 16 + lr, npos - 1);
            const int y = r_lo + p / O, x = p % O;
            f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
            if (XS) {
                // split operands (k_pnet conv1's K layout): slots 8*(lk&1) .. +7 of row ky are
                // pixels x + 2*(lk&1), +1; row 3 (s2 = 1, lk >= 2) has zero weights
                const _Float16* c0p = (const _Float16*)cp0;
                f32x4 d0 = c0, d1 = c0;
#pragma unroll
                for (int s2 = 0; s2 < 2; s2++) {
                    const int ky = min(2 * s2 + (lk >> 1), 2);
                    const int pix = (y + ky) * S + x + 2 * (lk & 1);
                    const f16x8 xa = ld_h8(c0p + pix * 4);
                    c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa, wh0[s2][0], c0, 0, 0, 0);
                    c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa, wh0[s2][1], c1, 0, 0, 0);
                    d0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa, wh1[s2][0], d0, 0, 0, 0);
                    d1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa, wh1[s2][1], d1, 0, 0, 0);
                    if (!exact) {
                        const f16x8 xb = ld_h8(c0p + (S * S + 1) * 4 + pix * 4);
                        d0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(xb, wh0[s2][0], d0, 0, 0, 0);
                        d1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(xb, wh0[s2][1], d1, 0, 0, 0);
                    }
                }
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    c0[i] = __builtin_fmaf(d0[i], 0.00048828125f, c0[i]);
                    c1[i] = __builtin_fmaf(d1[i], 0.00048828125f, c1[i]);
                }
            } else {
#pragma unroll
                for (int s = 0; s < 7; s++) {
                    const int kk = 4 * s + lk;
                    const int kc = min(kk, 26);
                    const int c = kc / 9, r = kc - 9 * c;
                    const float av = kk < 27 ? crop[c * S * S + (y + r / 3) * S + x + r % 3] : 0.f;
                    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, wb[s][0], c0, 0, 0, 0);
                    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(av, wb[s][1], c1, 0, 0, 0);
                }
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int q = f * 16 + 4 * lk + i;
                if (q < npos) {
                    const int yq = r_lo + q / O;
                    const int slot = (yq % BR) * O + (q - (yq - r_lo) * O);
                    cv[lr * CS + slot] = prelu(c0[i] + bb0, aa0);
                    cv[(16 + lr) * CS + slot] = prelu(c1[i] + bb1, aa1);
                }
            }
        }
        __syncthreads();
        const int npr = min(PB, P - pr0);
        bool bad = false;
        if (ovf) {
            // split-pair output (gemm_x3.hpp: 32-B chunks [x0 x 8 | x1 x 8] of 8 channels): one
            // thread per (pooled position, 8-channel chunk), two 16-B stores
            for (int i = tid; i < ((dbg & 4) ? 0 : npr * P * 4); i += NT) {
                const int cg = i & 3, t = i >> 2;
                const int px = t % P, pyl = t / P;
                int xo[3], yo[3];
#pragma unroll
                for (int d = 0; d < 3; d++) {
                    xo[d] = min(2 * px + d, O - 1);
                    yo[d] = (min(2 * (pr0 + pyl) + d, O - 1) % BR) * O;
                }
                f16x8 h0, h1;
#pragma unroll
                for (int c8 = 0; c8 < 8; c8++) {
                    const float* cr = cv + (8 * cg + c8) * CS;
                    float m = cr[yo[0] + xo[0]];
#pragma unroll
                    for (int dy = 0; dy < 3; dy++)
#pragma unroll
                        for (int dx = 0; dx < 3; dx++)
                            if (dy | dx) m = fmaxf(m, cr[yo[dy] + xo[dx]]);
                    h0[c8] = (_Float16)m;
                    h1[c8] = (_Float16)((m - (float)h0[c8]) * 2048.f);
                    bad |= !(fabsf(m) < 16384.f);
                }
                f16x8* ch = (f16x8*)(o + ((pr0 + pyl) * P + px) * 32 + 8 * cg);
                ch[0] = h0;
                ch[1] = h1;
            }
        }
        for (int i = tid; i < ((dbg & 4) || ovf ? 0 : npr * P * 32); i += NT) {
            const int c = i & 31, t = i >> 5;
            const int px = t % P, pyl = t / P;
            // ceil-mode windows clipped at the map edge: a clipped index is clamped onto the
            // window's last valid row / column instead (max is idempotent), so every lane runs
            // the same 9 reads
            const float* cr = cv + c * CS;
            int xo[3], yo[3];
#pragma unroll
            for (int d = 0; d < 3; d++) {
                xo[d] = min(2 * px + d, O - 1);
                yo[d] = (min(2 * (pr0 + pyl) + d, O - 1) % BR) * O;
            }
            float m = cr[yo[0] + xo[0]];
#pragma unroll
            for (int dy = 0; dy < 3; dy++)
#pragma unroll
                for (int dx = 0; dx < 3; dx++)
                    if (dy | dx) m = fmaxf(m, cr[yo[dy] + xo[dx]]);
            if (ovf) {
                // split-pair layout (gemm_x3.hpp) for the split-mode conv2: 32-B chunks of 8 channels
                // [x0 x 8 | x1 x 8]; a value beyond the fp16 range raises *ovf
                const _Float16 h0 = (_Float16)m, h1 = (_Float16)((m - (float)h0) * 2048.f);
                _Float16* ch = (_Float16*)(o + ((pr0 + pyl) * P + px) * 32 + (c & ~7));
                ch[c & 7] = h0;
                ch[8 + (c & 7)] = h1;
                bad |= !(fabsf(m) < 16384.f);
            } else {
                o[((pr0 + pyl) * P + px) * 32 + c] = m;
            }
        }
        if (ovf && __ballot(bad) && lane == 0) atomicOr(ovf, 1);
        __syncthreads();
    }
}

// RNet front (S = 24) as one WAVE per candidate, NWV candidates per workgroup, each wave on its own
// LDS slices with no workgroup barrier: the one-workgroup-per-candidate kernel above spends most of
// its ~46k cycles per candidate in dependent phases (box -> SAT gathers -> 4 bands of conv / pool,
// 8 barriers) that the few workgroups per CU do not overlap.  Same arithmetic, bit for bit: the
// crop's bin averages, conv1 on the split-fp16 16x16x32 MFMA chains (k_pnet conv1's K layout,
// cross terms 2^-11-scaled into the main chain), PReLU, the clamped ceil-mode 3x3/2 max-pool, the
// split-pair output and the fp16-range flag.  Conv rows go to a ring of 3 rows per channel (slot =
// row % 3); pooled row py needs conv rows 2 py .. 2 py + 2.
__device__ inline void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
template <int NWV>
__global__ __launch_bounds__(64 * NWV) void k_cand_front_w24(const void* __restrict__ sat, int pk, int H, int W,
                                                             const float4* __restrict__ boxes,
                                                             const int32_t* __restrict__ img, int64_t n,
                                                             const _Float16* __restrict__ w1h,
                                                             const float* __restrict__ b1, const float* __restrict__ a1,
                                                             float* __restrict__ out, int32_t* __restrict__ err,
                                                             int* __restrict__ ovf) {
    constexpr int S = 24, O = S - 2, P = (O - 3 + 1) / 2 + 1;  // 22, 11
    // conv ring: [3 rows x 22 columns][32 channels + 4 pad] fp32, channel-contiguous so the pool
    // reads 8 channels of a window position as two ds_read_b128 (72 scalar reads before)
    constexpr int RS = 36;
    typedef __attribute__((ext_vector_type(4))) _Float16 h4;
    __shared__ h4 crop_s[NWV][2][S * S + 1];
    __shared__ __attribute__((aligned(16))) float cv_s[NWV][3 * O * RS];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, lr = lane & 15, lk = lane >> 4;
    const int64_t k = (int64_t)blockIdx.x * NWV + wv;
    if (k >= n) return;  // (wave-uniform; no workgroup barrier below)
    h4* cp0 = crop_s[wv][0];
    h4* cp1 = crop_s[wv][1];
    float* cv = cv_s[wv];
    float* o = out + k * (P * P * 32);
    int y0, x0, hc, wc;
    if (!crop_rect(boxes[k], H, W, y0, x0, hc, wc)) {
        if (lane == 0) atomicAdd(err, 1);
        for (int i = lane; i < P * P * 32; i += 64) o[i] = 0.f;
        return;
    }
    const bool exact = hc <= S && wc <= S;
    if (lane == 0) {
        const h4 z = {(_Float16)0.f, (_Float16)0.f, (_Float16)0.f, (_Float16)0.f};
        cp0[S * S] = z;
        cp1[S * S] = z;
    }
    // crop: 9 pixels per lane in 3 rounds of 3 (12 SAT corner loads in flight per round)
    const int64_t sk = (int64_t)img[k] * (H + 1) * (W + 1);
#pragma unroll
    for (int rd = 0; rd < 3; rd++) {
        int idx[3], kh[3], kw[3];
        int3 sm[3];
#pragma unroll
        for (int j = 0; j < 3; j++) idx[j] = lane + 64 * (3 * rd + j);
        if (pk)
            crop_bins<3, S, true>(sat, sk, W + 1, y0, x0, hc, wc, idx, sm, kh, kw);
        else
            crop_bins<3, S, false>(sat, sk, W + 1, y0, x0, hc, wc, idx, sm, kh, kw);
#pragma unroll
        for (int j = 0; j < 3; j++) {
            const int i = idx[j];
            _Float16 r0, r1, g0, g1, c0, c1;
            split_f16(bin_avg(sm[j].x, kh[j], kw[j]), r0, r1);
            split_f16(bin_avg(sm[j].y, kh[j], kw[j]), g0, g1);
            split_f16(bin_avg(sm[j].z, kh[j], kw[j]), c0, c1);
            cp0[i] = h4{r0, g0, c0, (_Float16)0.f};
            if (!exact) cp1[i] = h4{r1, g1, c1, (_Float16)0.f};
        }
    }
    // conv1 weights: split planes [2][32][64] as the B operand, channel block nb = co / 16
    f16x8 wh0[2][2], wh1[2][2];
#pragma unroll
    for (int s2 = 0; s2 < 2; s2++)
#pragma unroll
        for (int nb = 0; nb < 2; nb++) {
            const _Float16* src = w1h + (16 * nb + lr) * 64 + 32 * s2 + 8 * lk;
            wh0[s2][nb] = *(const f16x8*)src;
            wh1[s2][nb] = *(const f16x8*)(src + 32 * 64);
        }
    const float bb0 = b1[lr], bb1 = b1[16 + lr], aa0 = a1[lr], aa1 = a1[16 + lr];
    wave_sync();
    const _Float16* c0p = (const _Float16*)cp0;
    bool bad = false;
    for (int py = 0; py < P; py++) {
        // conv rows [r_lo, r_hi] into the ring (row 2 py is the previous pooled row's last)
        const int r_lo = py == 0 ? 0 : 2 * py + 1, r_hi = min(2 * py + 2, O - 1);
        const int npos = (r_hi - r_lo + 1) * O;
        for (int f = 0; f * 16 < npos; f++) {
            const int p = min(f * 16 + lr, npos - 1);
            const int y = r_lo + p / O, x = p % O;
            f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = c0, d0 = c0, d1 = c0;
#pragma unroll
            for (int s2 = 0; s2 < 2; s2++) {
                const int ky = min(2 * s2 + (lk >> 1), 2);
                const int pix = (y + ky) * S + x + 2 * (lk & 1);
                const f16x8 xa = ld_h8(c0p + pix * 4);
                c0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa, wh0[s2][0], c0, 0, 0, 0);
                c1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa, wh0[s2][1], c1, 0, 0, 0);
                d0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa, wh1[s2][0], d0, 0, 0, 0);
                d1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(xa, wh1[s2][1], d1, 0, 0, 0);
                if (!exact) {
                    const f16x8 xb = ld_h8(c0p + (S * S + 1) * 4 + pix * 4);
                    d0 = __builtin_amdgcn_mfma_f32_16x16x32_f16(xb, wh0[s2][0], d0, 0, 0, 0);
                    d1 = __builtin_amdgcn_mfma_f32_16x16x32_f16(xb, wh0[s2][1], d1, 0, 0, 0);
                }
            }
#pragma unroll
            for (int i = 0; i < 4; i++) {
                const int q = f * 16 + 4 * lk + i;
                if (q < npos) {
                    const int yq = r_lo + q / O;
                    const int slot = (yq % 3) * O + (q - (yq - r_lo) * O);
                    cv[slot * RS + lr] = prelu(__builtin_fmaf(d0[i], 0.00048828125f, c0[i]) + bb0, aa0);
                    cv[slot * RS + 16 + lr] = prelu(__builtin_fmaf(d1[i], 0.00048828125f, c1[i]) + bb1, aa1);
                }
            }
        }
        wave_sync();
        // pooled row py: 11 columns x 4 chunks of 8 channels (44 lanes), split-pair 32-B chunks
        if (lane < P * 4) {
            const int cg = lane & 3, px = lane >> 2;
            int xo[3], yo[3];
#pragma unroll
            for (int d = 0; d < 3; d++) {
                xo[d] = min(2 * px + d, O - 1);
                yo[d] = (min(2 * py + d, O - 1) % 3) * O;
            }
            f16x8 h0, h1;
            float m[8];
#pragma unroll
            for (int dy = 0; dy < 3; dy++)
#pragma unroll
                for (int dx = 0; dx < 3; dx++) {
                    const float* cr = cv + (yo[dy] + xo[dx]) * RS + 8 * cg;
                    const f32x4 lo = *(const f32x4*)cr, hi = *(const f32x4*)(cr + 4);
#pragma unroll
                    for (int c = 0; c < 4; c++) {
                        // (the same max order per channel as the scalar version: (0,0) first)
                        m[c] = (dy | dx) ? fmaxf(m[c], lo[c]) : lo[c];
                        m[4 + c] = (dy | dx) ? fmaxf(m[4 + c], hi[c]) : hi[c];
                    }
                }
#pragma unroll
            for (int c8 = 0; c8 < 8; c8++) {
                h0[c8] = (_Float16)m[c8];
                h1[c8] = (_Float16)((m[c8] - (float)h0[c8]) * 2048.f);
                bad |= !(fabsf(m[c8]) < 16384.f);
            }
            f16x8* ch = (f16x8*)(o + (py * P + px) * 32 + 8 * cg);
            ch[0] = h0;
            ch[1] = h1;
        }
        wave_sync();  // the ring rows are rewritten by the next pooled row
    }
    if (__ballot(bad) && lane == 0) atomicOr(ovf, 1);
}

int cand_front_side(bool onet) { return onet ? 23 : 11; }

// RNet front as one wave per candidate (1, default) or one workgroup per candidate (VTF_FRONT_WAVE=0);
// read per launch (the tests run both)
static bool wave_front() {
    const char* e = std::getenv("VTF_FRONT_WAVE");
    return !(e && std::atoi(e) == 0);
}

void launch_cand_front(bool onet, const void* sat, int pk, int H, int W, const float4* boxes, const int32_t* img,
                       int64_t n, const float* w1, const _Float16* w1h, const float* b1, const float* a1, float* out,
                       int32_t* err, hipStream_t st, int* ovf) {
    if (n <= 0) return;
    static const int dbg = [] {  // phase-skip mask for profiling (VTF_FRONT_DEBUG): 1 crop, 2 conv1, 4 pool
        const char* e = std::getenv("VTF_FRONT_DEBUG");
        return e ? std::atoi(e) : 0;
    }();
    // pool rows per band of the ONet front (VTF_FRONT_PB = 1 / 2 / 3): more rows per band = fewer
    // barriers and more conv fragments per band for the 8 waves, against a larger conv ring
    // (78 KB at 3: two workgroups per CU either way); 3 measured 441 -> 402 us per det-batch
    const char* pbe = std::getenv("VTF_FRONT_PB");
    const int pb = pbe ? std::atoi(pbe) : 3;
    // w1h (split conv1 planes) selects conv1 on fp16 matrix cores; null keeps the fp32 MFMA path
    if (onet && w1h && pb == 2)
        k_cand_front<48, 2, 512, true><<<(unsigned)n, 512, 0, st>>>(sat, pk, H, W, boxes, img, w1, w1h, b1, a1, out, err, dbg, ovf);
    else if (onet && w1h && pb == 3)
        k_cand_front<48, 3, 512, true><<<(unsigned)n, 512, 0, st>>>(sat, pk, H, W, boxes, img, w1, w1h, b1, a1, out, err, dbg, ovf);
    else if (onet && w1h)
        k_cand_front<48, 1, 512, true><<<(unsigned)n, 512, 0, st>>>(sat, pk, H, W, boxes, img, w1, w1h, b1, a1, out, err, dbg, ovf);
    else if (onet)
        k_cand_front<48, 1, 512, false><<<(unsigned)n, 512, 0, st>>>(sat, pk, H, W, boxes, img, w1, w1h, b1, a1, out, err, dbg, ovf);
    else if (w1h && ovf && wave_front() && !dbg)
        k_cand_front_w24<4><<<(unsigned)cdiv(n, 4), 256, 0, st>>>(sat, pk, H, W, boxes, img, n, w1h, b1, a1, out, err, ovf);
    else if (w1h)
        k_cand_front<24, 3, 256, true><<<(unsigned)n, 256, 0, st>>>(sat, pk, H, W, boxes, img, w1, w1h, b1, a1, out, err, dbg, ovf);
    else
        k_cand_front<24, 3, 256, false><<<(unsigned)n, 256, 0, st>>>(sat, pk, H, W, boxes, img, w1, w1h, b1, a1, out, err, dbg, ovf);
}

// heads: x [n, D] -> softmax(x W1^T + b1)[:, 1], x W2^T + b2 (4), optional x W3^T + b3 (10).
// One wave per candidate; lanes split D, wave-reduced.  RNet's softmax is over the last dim
// (torch multiplies by the reciprocal sum), ONet's too.
__global__ __launch_bounds__(64) void k_heads(const float* __restrict__ x, int64_t n, int D,
                                              const float* __restrict__ w1, const float* __restrict__ b1,
                                              const float* __restrict__ w2, const float* __restrict__ b2,
                                              const float* __restrict__ w3, const float* __restrict__ b3,
                                              float* __restrict__ prob, float4* __restrict__ reg,
                                              float* __restrict__ lm) {
    const int64_t k = blockIdx.x;
    const int lane = threadIdx.x;
    const float* xk = x + k * D;
    float part[16];
#pragma unroll
    for (int j = 0; j < 16; j++) part[j] = 0.f;
    for (int d = lane; d < D; d += 64) {
        float f = xk[d];
        part[0] = fmaf(f, w1[d], part[0]);
        part[1] = fmaf(f, w1[D + d], part[1]);
#pragma unroll
        for (int j = 0; j < 4; j++) part[2 + j] = fmaf(f, w2[j * D + d], part[2 + j]);
        if (w3) {
#pragma unroll
            for (int j = 0; j < 10; j++) part[6 + j] = fmaf(f, w3[j * D + d], part[6 + j]);
        }
    }
#pragma unroll
    for (int j = 0; j < 16; j++)
        for (int off = 32; off > 0; off >>= 1) part[j] += __shfl_xor(part[j], off);
    if (lane == 0) {
        float a0 = part[0] + b1[0], a1 = part[1] + b1[1];
        float mx = fmaxf(a0, a1);
        float e0 = expf(a0 - mx), e1 = expf(a1 - mx);
        prob[k] = e1 * __fdiv_rn(1.0f, e0 + e1);
        reg[k] = make_float4(part[2] + b2[0], part[3] + b2[1], part[4] + b2[2], part[5] + b2[3]);
        if (w3)
            for (int j = 0; j < 10; j++) lm[k * 10 + j] = part[6 + j] + b3[j];
    }
}

void launch_heads(const float* x, int64_t n, int D, const float* w1, const float* b1, const float* w2,
                  const float* b2, const float* w3, const float* b3, float* prob, float4* reg, float* lm,
                  hipStream_t st) {
    if (n > 0) k_heads<<<(unsigned)n, 64, 0, st>>>(x, n, D, w1, b1, w2, b2, w3, b3, prob, reg, lm);
}

// ----------------------------------------------------------------------------------- box ops

// stage-1 decode of sorted candidates: (level, lin) -> box, score, img, reg (mtcnn.py:183-194)
__global__ void k_decode_stage1(const uint64_t* __restrict__ key_sorted, const int32_t* __restrict__ slot_sorted,
                                const float* __restrict__ score, const float4* __restrict__ regv,
                                const PNetLevel* __restrict__ lv, int64_t n, float4* __restrict__ boxes,
                                float* __restrict__ sc, float4* __restrict__ reg, int32_t* __restrict__ img,
                                int32_t* __restrict__ call) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    uint64_t key = key_sorted[k];
    int L = (int)(key >> 32);
    uint32_t lin = (uint32_t)key;
    const PNetLevel P = lv[L];
    uint32_t plane = (uint32_t)P.ph * (uint32_t)P.pw;
    int b = (int)(lin / plane);
    uint32_t cell = lin % plane;
    int h = (int)(cell / P.pw), wcol = (int)(cell % P.pw);
    float s = P.scale;
    // q1 = floor((2*bb + 1) / s), q2 = floor((2*bb + 12) / s): int64 tensor / python float -> fp32
    float4 bx;
    bx.x = floorf(__fdiv_rn((float)(2 * wcol + 1), s));
    bx.y = floorf(__fdiv_rn((float)(2 * h + 1), s));
    bx.z = floorf(__fdiv_rn((float)(2 * wcol + 12), s));
    bx.w = floorf(__fdiv_rn((float)(2 * h + 12), s));
    int32_t slot = slot_sorted[k];
    boxes[k] = bx;
    sc[k] = score[slot];
    reg[k] = regv[slot];
    img[k] = b;
    call[k] = L;
}

// gather by index list, then optional refine (mtcnn.py:254-262) + square (264-271)
__global__ void k_gather_refine(const int32_t* __restrict__ idx, int64_t n, const float4* __restrict__ bin,
                                const float* __restrict__ sin, const float4* __restrict__ rin,
                                const int32_t* __restrict__ iin, int refine, int plus_one, int square,
                                float4* __restrict__ bout, float* __restrict__ sout, float4* __restrict__ rout,
                                int32_t* __restrict__ iout, int32_t* __restrict__ zout, int32_t* __restrict__ zw, int nzw) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    // folded memsets: zout[k] = 0 (the next NMS's call ids), zw[0..nzw) = 0 (stage guards / error
    // counters) -- one launch instead of a fill kernel each
    if (k < nzw) zw[k] = 0;
    if (k >= n) return;
    if (zout) zout[k] = 0;
    int32_t e = idx ? idx[k] : (int32_t)k;
    float4 b = bin[e];
    float4 r = rin ? rin[e] : make_float4(0.f, 0.f, 0.f, 0.f);
    if (refine) {
        float w = b.z - b.x, h = b.w - b.y;
        if (plus_one) {
            w = w + 1.0f;
            h = h + 1.0f;
        }
        float4 o;
        o.x = b.x + r.x * w;
        o.y = b.y + r.y * h;
        o.z = b.z + r.z * w;
        o.w = b.w + r.w * h;
        b = o;
    }
    if (square) {
        float h = b.w - b.y, w = b.z - b.x;
        float l = fmaxf(w, h);
        b.x = (b.x + w * 0.5f) - l * 0.5f;
        b.y = (b.y + h * 0.5f) - l * 0.5f;
        b.z = b.x + l;
        b.w = b.y + l;
    }
    bout[k] = b;
    if (sout) sout[k] = sin[e];
    if (rout) rout[k] = r;
    if (iout) iout[k] = iin[e];
}

// flag[k] = score[k] > thr (fp32 compare)
__global__ void k_threshold(const float* __restrict__ s, int64_t n, float thr, int32_t* __restrict__ flag) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n) flag[k] = s[k] > thr ? 1 : 0;
}

__global__ void k_flag_compact(const int32_t* __restrict__ flag, const int32_t* __restrict__ incl, int64_t n,
                               int32_t* __restrict__ out, int32_t* __restrict__ mail, const int32_t* __restrict__ ctl,
                               int nctl) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n && flag[k]) out[incl[k] - 1] = (int32_t)k;
    // the count (and the stage's control words) straight to the host mailbox: read after the
    // stream sync, no blit copy
    if (mail && k == n - 1) {
        mail[0] = incl[n - 1];
        for (int i = 0; i < nctl; i++) mail[1 + i] = ctl[i];
    }
}

// landmarks from pre-refine boxes (mtcnn.py:235-239): out [n][5][2]
__global__ void k_landmarks(const float4* __restrict__ boxes, const float* __restrict__ lm, int64_t n,
                            float* __restrict__ out) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    float4 b = boxes[k];
    float w = (b.z - b.x) + 1.0f, h = (b.w - b.y) + 1.0f;
    for (int j = 0; j < 5; j++) {
        out[k * 10 + 2 * j] = (w * lm[k * 10 + j] + b.x) - 1.0f;
        out[k * 10 + 2 * j + 1] = (h * lm[k * 10 + 5 + j] + b.y) - 1.0f;
    }
}

// _nms_vectorized(method='Min', chain_suppression=True) (mtcnn.py:273-309) on score-sorted
// rows: drop row k if any earlier row of the same image overlaps it with IoM > thr.
// earlier boxes (in `order`) staged through LDS in tiles of IOM_TILE; each row is scanned by
// IOM_SUB adjacent lanes (interleaved predecessors), their drop flags OR-ed at the end
constexpr int IOM_TILE = 1024, IOM_SUB = 4, IOM_ROWS = 256 / IOM_SUB;
__global__ __launch_bounds__(256) void k_iom_chain(const float4* __restrict__ boxes, const int32_t* __restrict__ img,
                                                   const int32_t* __restrict__ order, int64_t n, float thr,
                                                   int32_t* __restrict__ keep) {
    __shared__ float4 sb[IOM_TILE];
    __shared__ int32_t si[IOM_TILE];
    const int sub = threadIdx.x % IOM_SUB;
    const int64_t k = (int64_t)blockIdx.x * IOM_ROWS + threadIdx.x / IOM_SUB;
    const bool valid = k < n;
    float4 b2 = make_float4(0.f, 0.f, 0.f, 0.f);
    int32_t ij = -1;
    if (valid) {
        const int32_t j = order[k];
        b2 = boxes[j];
        ij = img[j];
    }
    const float a2 = ((b2.z - b2.x) + 1.0f) * ((b2.w - b2.y) + 1.0f);
    int drop = 0;
    const int64_t last = min(n, ((int64_t)blockIdx.x + 1) * IOM_ROWS);  // this block's rows are < last
    for (int64_t q0 = 0; q0 < last - 1; q0 += IOM_TILE) {
        __syncthreads();
        for (int t = threadIdx.x; t < IOM_TILE; t += blockDim.x)
            if (q0 + t < n) {
                const int32_t i = order[q0 + t];
                sb[t] = boxes[i];
                si[t] = img[i];
            }
        __syncthreads();
        const int64_t qe = valid ? min((int64_t)IOM_TILE, k - q0) : 0;
        for (int t = sub; t < qe && !drop; t += IOM_SUB) {
            if (si[t] != ij) continue;
            const float4 b1 = sb[t];
            const float iw = (fminf(b1.z, b2.z) - fmaxf(b1.x, b2.x)) + 1.0f;
            const float ih = (fminf(b1.w, b2.w) - fmaxf(b1.y, b2.y)) + 1.0f;
            if (!(iw > 0.f && ih > 0.f)) continue;
            const float inter = iw * ih;
            const float a1 = ((b1.z - b1.x) + 1.0f) * ((b1.w - b1.y) + 1.0f);
            const float iom = __fdiv_rn(inter, fminf(a1, a2));
            if (iom > thr) drop = 1;
        }
    }
    drop |= __shfl_xor(drop, 1);
    drop |= __shfl_xor(drop, 2);
    if (valid && sub == 0) keep[k] = !drop;
}

void launch_decode_stage1(const uint64_t* key_sorted, const int32_t* slot_sorted, const float* score,
                          const float4* regv, const PNetLevel* lv, int64_t n, float4* boxes, float* sc, float4* reg,
                          int32_t* img, int32_t* call, hipStream_t st) {
    if (n > 0)
        k_decode_stage1<<<cdiv(n, 256), 256, 0, st>>>(key_sorted, slot_sorted, score, regv, lv, n, boxes, sc, reg,
                                                       img, call);
}
void launch_gather_refine(const int32_t* idx, int64_t n, const float4* bin, const float* sin, const float4* rin,
                          const int32_t* iin, int refine, int plus_one, int square, float4* bout, float* sout,
                          float4* rout, int32_t* iout, hipStream_t st, int32_t* zout, int32_t* zw, int nzw) {
    VTF_CHECK(nzw >= 0 && nzw <= 256, VTF_E_ARG, "gather_refine: at most 256 zeroed words");
    if (n > 0 || nzw > 0)
        k_gather_refine<<<std::max(1, cdiv(n, 256)), 256, 0, st>>>(idx, n, bin, sin, rin, iin, refine, plus_one, square,
                                                                    bout, sout, rout, iout, zout, zw, nzw);
}
void launch_threshold(const float* s, int64_t n, float thr, int32_t* flag, hipStream_t st) {
    if (n > 0) k_threshold<<<cdiv(n, 256), 256, 0, st>>>(s, n, thr, flag);
}
void launch_flag_compact(const int32_t* flag, const int32_t* incl, int64_t n, int32_t* out, hipStream_t st,
                         int32_t* mail, const int32_t* ctl, int nctl) {
    if (n > 0) k_flag_compact<<<cdiv(n, 256), 256, 0, st>>>(flag, incl, n, out, mail, ctl, nctl);
}
void launch_landmarks(const float4* boxes, const float* lm, int64_t n, float* out, hipStream_t st) {
    if (n > 0) k_landmarks<<<cdiv(n, 256), 256, 0, st>>>(boxes, lm, n, out);
}
void launch_iom_chain(const float4* boxes, const int32_t* img, const int32_t* order, int64_t n, float thr,
                      int32_t* keep, hipStream_t st) {
    if (n > 0) k_iom_chain<<<cdiv(n, IOM_ROWS), 256, 0, st>>>(boxes, img, order, n, thr, keep);
}

}  // namespace vtf

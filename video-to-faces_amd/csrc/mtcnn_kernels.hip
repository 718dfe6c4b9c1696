// MTCNN kernels for gfx950 (fp32; parity with the reference PyTorch-CPU path).
//
// Reference: src/videotofaces/detectors/mtcnn.py
//   _preprocess 133-139, _resample 150-151, PNet 12-38, stage-1 candidates 183-194,
//   _get_cropped_candidates 153-163, RNet 41-76, ONet 79-121.
//
// MI355X design:
//   * k_pnet: ONE launch per det-batch covers every pyramid level of every frame.  Each
//     256-thread workgroup owns a 16x32 tile of PNet output cells.  The level pixels it
//     needs (42x74x3) are computed on the fly from the uint8 BGR frame (preprocess +
//     adaptive_avg_pool2d, bit-exact: exact (u-127.5)/128, row-major fp32 bin sum, /kh, /kw)
//     straight into LDS, so the 10.7 Mpx/frame pyramid never exists in HBM.  conv1+PReLU+
//     maxpool(ceil), conv2+PReLU, conv3+PReLU and both 1x1 heads + softmax run from LDS with
//     weights streamed through the scalar cache (wave-uniform, transposed to [ci][ky][kx][co]
//     on the host so one s_load_dwordx16 feeds 16 v_fma).  Cells with p >= 0.6 are appended
//     with one wave-aggregated atomic -- the dense prob/reg maps are never written.
//   * k_rnet / k_onet: one workgroup per candidate box; the crop + adaptive pool to 24x24 /
//     48x48 (replacing the reference's per-box Python loop) feeds the whole network in LDS.
// Build with -ffp-contract=off: only explicit fmaf() fuses.
#include <algorithm>

#include "common.hpp"
#include "mtcnn.hpp"

namespace vtf {

typedef __attribute__((ext_vector_type(4))) float f32x4;

// ----------------------------------------------------------------------------------- helpers

// Level pixel (RGB channel c) of MTCNN._resample(_preprocess(frames)), from uint8 BGR.
__device__ inline float level_value(const uint8_t* __restrict__ fr, int64_t row_stride, int c, int ly, int lx,
                                    int H, int W, int lh, int lw) {
    int y0 = (int)(((int64_t)ly * H) / lh);
    int y1 = (int)(((int64_t)(ly + 1) * H + lh - 1) / lh);
    int x0 = (int)(((int64_t)lx * W) / lw);
    int x1 = (int)(((int64_t)(lx + 1) * W + lw - 1) / lw);
    const uint8_t* p = fr + (2 - c);
    float s = 0.f;
    for (int y = y0; y < y1; y++) {
        const uint8_t* r = p + (int64_t)y * row_stride;
        for (int x = x0; x < x1; x++) s = s + ((float)r[x * 3] - 127.5f) * 0.0078125f;
    }
    return __fdiv_rn(__fdiv_rn(s, (float)(y1 - y0)), (float)(x1 - x0));
}

// Crop [y0, y0+hc) x [x0, x0+wc) of the preprocessed frame adaptive-pooled to S x S.
__device__ inline float crop_value(const uint8_t* __restrict__ fr, int64_t row_stride, int c, int r, int q,
                                   int y0c, int x0c, int hc, int wc, int S) {
    int ys = (r * hc) / S, ye = ((r + 1) * hc + S - 1) / S;
    int xs = (q * wc) / S, xe = ((q + 1) * wc + S - 1) / S;
    const uint8_t* p = fr + (2 - c);
    float s = 0.f;
    for (int y = ys; y < ye; y++) {
        const uint8_t* row = p + (int64_t)(y0c + y) * row_stride;
        for (int x = xs; x < xe; x++) s = s + ((float)row[(x0c + x) * 3] - 127.5f) * 0.0078125f;
    }
    return __fdiv_rn(__fdiv_rn(s, (float)(ye - ys)), (float)(xe - xs));
}

__device__ inline float prelu(float x, float a) { return x > 0.f ? x : a * x; }

// Python int() of a float, saturated (values beyond +-2e9 only matter through clamping).
__device__ inline int trunc_sat(float v) {
    v = fminf(fmaxf(v, -2.0e9f), 2.0e9f);
    return (int)v;
}

// _get_cropped_candidates box -> crop rect; false if the reference would skip the box.
__device__ inline bool crop_rect(float4 b, int H, int W, int& y0, int& x0, int& hc, int& wc) {
    int ix1 = max(1, trunc_sat(b.x)), iy1 = max(1, trunc_sat(b.y));
    int ix2 = min(W, trunc_sat(b.z)), iy2 = min(H, trunc_sat(b.w));
    if (!(iy2 > iy1 - 1 && ix2 > ix1 - 1)) return false;
    y0 = iy1 - 1;
    x0 = ix1 - 1;
    hc = iy2 - y0;
    wc = ix2 - x0;
    return true;
}

// constant-address-space views of the weight structs (scalar loads, see common.hpp)
#define CW const VTF_CONST float*
struct PNetWC { CW c1w; CW c1b; CW p1; CW c2w; CW c2b; CW p2; CW c3w; CW c3b; CW p3; CW c41w; CW c41b; CW c42w; CW c42b; };
struct RNetWC { CW c1w; CW c1b; CW p1; CW c2w; CW c2b; CW p2; CW c3w; CW c3b; CW p3; CW d4w; CW d4b; CW p4; CW d51w; CW d51b; CW d52w; CW d52b; };
struct ONetWC { CW c1w; CW c1b; CW p1; CW c2w; CW c2b; CW p2; CW c3w; CW c3b; CW p3; CW c4w; CW c4b; CW p4; CW d5w; CW d5b; CW p5; CW d61w; CW d61b; CW d62w; CW d62b; CW d63w; CW d63b; };
#undef CW
__device__ inline PNetWC to_const(const PNetW& w) {
    return {cptr(w.c1w), cptr(w.c1b), cptr(w.p1), cptr(w.c2w), cptr(w.c2b), cptr(w.p2), cptr(w.c3w), cptr(w.c3b),
            cptr(w.p3), cptr(w.c41w), cptr(w.c41b), cptr(w.c42w), cptr(w.c42b)};
}
__device__ inline RNetWC to_const(const RNetW& w) {
    return {cptr(w.c1w), cptr(w.c1b), cptr(w.p1), cptr(w.c2w), cptr(w.c2b), cptr(w.p2), cptr(w.c3w), cptr(w.c3b),
            cptr(w.p3), cptr(w.d4w), cptr(w.d4b), cptr(w.p4), cptr(w.d51w), cptr(w.d51b), cptr(w.d52w), cptr(w.d52b)};
}
__device__ inline ONetWC to_const(const ONetW& w) {
    return {cptr(w.c1w), cptr(w.c1b), cptr(w.p1),  cptr(w.c2w),  cptr(w.c2b),  cptr(w.p2),  cptr(w.c3w),
            cptr(w.c3b), cptr(w.p3),  cptr(w.c4w), cptr(w.c4b),  cptr(w.p4),   cptr(w.d5w), cptr(w.d5b),
            cptr(w.p5),  cptr(w.d61w), cptr(w.d61b), cptr(w.d62w), cptr(w.d62b), cptr(w.d63w), cptr(w.d63b)};
}

// ----------------------------------------------------------------------------------- resample

__global__ void k_resample(const uint8_t* __restrict__ frames, int64_t frame_stride, int64_t row_stride, int B,
                           int H, int W, int lh, int lw, float* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    int64_t n = (int64_t)B * 3 * lh * lw;
    if (i >= n) return;
    int lx = (int)(i % lw);
    int ly = (int)((i / lw) % lh);
    int c = (int)((i / ((int64_t)lw * lh)) % 3);
    int b = (int)(i / ((int64_t)lw * lh * 3));
    out[i] = level_value(frames + (int64_t)b * frame_stride, row_stride, c, ly, lx, H, W, lh, lw);
}

void launch_resample(const uint8_t* frames, int64_t frame_stride, int64_t row_stride, int B, int H, int W, int lh,
                     int lw, float* out, hipStream_t st) {
    int64_t n = (int64_t)B * 3 * lh * lw;
    k_resample<<<cdiv(n, 256), 256, 0, st>>>(frames, frame_stride, row_stride, B, H, W, lh, lw, out);
}

// ----------------------------------------------------------------------------------- PNet

constexpr int PT_H = 16, PT_W = 32;                   // output cells per tile
constexpr int PL_H = 2 * PT_H + 10, PL_W = 2 * PT_W + 10;  // level tile 42 x 74
constexpr int PP_H = PT_H + 4, PP_W = PT_W + 4;       // pooled 20 x 36
constexpr int PC_H = PT_H + 2, PC_W = PT_W + 2;       // conv2 out 18 x 34
constexpr int P_LVL = 3 * PL_H * PL_W;                // 9324
constexpr int P_C2 = 16 * PC_H * PC_W;                // 9792
constexpr int P_POOL = 10 * PP_H * PP_W;              // 7200
constexpr int P_A = P_C2 > P_LVL ? P_C2 : P_LVL;

// exact x / k for the bin averages: power-of-two k is an exact multiply (bit-identical to the
// IEEE division), other k take the correctly-rounded division
__device__ inline float div_bin(float x, int k) {
    return (k & (k - 1)) == 0 ? x * __int_as_float((127 - __builtin_ctz(k)) << 23) : __fdiv_rn(x, (float)k);
}

constexpr int PNET_GROUPS_PER_CU = 2;
constexpr int PATCH_BYTES = P_POOL * 4;  // frame patch staged in the (not yet used) pooled buffer

template <bool DENSE>
__global__ __launch_bounds__(256, 2) void k_pnet(const uint8_t* __restrict__ frames, int64_t frame_stride,
                                                 int64_t row_stride, int H, int W,
                                                 const PNetLevel* __restrict__ lv, int n_levels,
                                                 int64_t total_tiles, uint32_t* __restrict__ tile_ctr, PNetW wg,
                                                 PNetOut o) {
    const auto wc = to_const(wg);
    __shared__ float sA[P_A];     // level tile, later conv2 output
    __shared__ float sP[P_POOL];  // frame patch (u8) during the fill, then pooled conv1
    __shared__ int2 ybin[PL_H], xbin[PL_W];
    __shared__ int s_tile;
    const int tid = threadIdx.x;
    const int lane = tid & 63, wave = tid >> 6;
    const int lr = lane & 15, lk = lane >> 4;

    // ---- weights and im2col offsets, loaded once per persistent workgroup
    float w1[7];
#pragma unroll
    for (int s = 0; s < 7; s++) {
        int k = 4 * s + lk;
        w1[s] = (k < 27 && lr < 10) ? wc.c1w[k * 10 + lr] : 0.f;
    }
    const float b1 = lr < 10 ? wc.c1b[lr] : 0.f, a1 = lr < 10 ? wc.p1[lr] : 0.f;
    const float b2 = wc.c2b[lr], a2 = wc.p2[lr];
    for (;;) {
        // ---- fetch the next tile (dynamic: pyramid tiles differ in cost)
        if (tid == 0) s_tile = (int)atomicAdd(tile_ctr, 1u);
        __syncthreads();
        const int64_t blk = s_tile;
        if (blk >= total_tiles) break;
        int L = 0;
        while (L + 1 < n_levels && blk >= lv[L + 1].tile_beg) L++;
        const PNetLevel P = lv[L];
        const int64_t t = blk - P.tile_beg;
        const int tiles_per_img = P.tiles_x * P.tiles_y;
        const int b = (int)(t / tiles_per_img);
        const int tt = (int)(t % tiles_per_img);
        const int oy0 = (tt / P.tiles_x) * PT_H, ox0 = (tt % P.tiles_x) * PT_W;
        const uint8_t* fr = frames + (int64_t)b * frame_stride;
        const int L1h = P.lh - 2, L1w = P.lw - 2;

        // ---- 1. level tile (rows 2*oy0 .. +42, cols 2*ox0 .. +74) = MTCNN._resample of the
        //         preprocessed frame, bit-exact; zero outside the level.
        if (tid < PL_H) {
            int ly = 2 * oy0 + tid;
            ybin[tid] = ly < P.lh ? make_int2((ly * H) / P.lh, ((ly + 1) * H + P.lh - 1) / P.lh) : make_int2(0, 0);
        } else if (tid < PL_H + PL_W) {
            int q = tid - PL_H, lx = 2 * ox0 + q;
            xbin[q] = lx < P.lw ? make_int2((lx * W) / P.lw, ((lx + 1) * W + P.lw - 1) / P.lw) : make_int2(0, 0);
        }
        __syncthreads();
        // frame patch covering every bin of the tile; staged to LDS with coalesced loads when it fits
        int fy0 = ybin[0].x, fx0 = xbin[0].x, fy1 = fy0, fx1 = fx0;
        {
            int ry = min(PL_H - 1, P.lh - 1 - 2 * oy0), rx = min(PL_W - 1, P.lw - 1 - 2 * ox0);
            fy1 = ybin[ry].y;
            fx1 = xbin[rx].y;
        }
        const int pw3 = (fx1 - fx0) * 3;
        const bool staged = !P.pre && (int64_t)(fy1 - fy0) * pw3 <= PATCH_BYTES;
        uint8_t* patch = (uint8_t*)sP;
        if (staged) {
            const int nbytes = (fy1 - fy0) * pw3;
            for (int i = tid; i < nbytes; i += 256) {
                int r = i / pw3, q = i - r * pw3;
                patch[i] = fr[(int64_t)(fy0 + r) * row_stride + fx0 * 3 + q];
            }
        }
        __syncthreads();
        if (P.pre) {
            // large-bin level precomputed by k_resample (bit-identical values)
            const float* pre = P.pre + (int64_t)b * 3 * P.lh * P.lw;
            for (int i = tid; i < ((o.dbg & 1) ? 0 : P_LVL); i += 256) {
                int c = i / (PL_H * PL_W), rq = i - c * (PL_H * PL_W);
                int r = rq / PL_W, q = rq - r * PL_W;
                int ly = 2 * oy0 + r, lx = 2 * ox0 + q;
                sA[i] = (ly < P.lh && lx < P.lw) ? pre[((int64_t)c * P.lh + ly) * P.lw + lx] : 0.f;
            }
        }
        for (int i = tid; i < ((o.dbg & 1) || P.pre ? 0 : PL_H * PL_W); i += 256) {
            int r = i / PL_W, q = i - r * PL_W;
            int2 yb = ybin[r], xb = xbin[q];
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
            sA[i] = in ? div_bin(div_bin(s0, kh), kw) : 0.f;
            sA[PL_H * PL_W + i] = in ? div_bin(div_bin(s1, kh), kw) : 0.f;
            sA[2 * PL_H * PL_W + i] = in ? div_bin(div_bin(s2, kh), kw) : 0.f;
        }
        __syncthreads();

        // ---- 2. conv1 (3->10, 3x3) + PReLU + maxpool 2x2 ceil on MFMA.  A row r of fragment
        //         f is conv1 position (2py+dy, 2px+dx) of pooled cell pp = 4f + r/4, corner r%4,
        //         so each lane's 4 accumulators (rows 4*lk..4*lk+3) ARE one pooling window.
        {
            constexpr int NPP = PP_H * PP_W;  // 720 pooled cells
            constexpr int NF1 = NPP / 4;      // 180 fragments
            const int corner = lr & 3, dy = corner >> 1, dx = corner & 1;
            for (int f0 = wave; f0 < ((o.dbg & 2) ? 0 : NF1); f0 += 8) {
                const int f1 = f0 + 4;
                const bool two = f1 < NF1;
                int pp0 = f0 * 4 + (lr >> 2), pp1 = (two ? f1 : f0) * 4 + (lr >> 2);
                int ab0 = (2 * (pp0 / PP_W) + dy) * PL_W + 2 * (pp0 % PP_W) + dx;
                int ab1 = (2 * (pp1 / PP_W) + dy) * PL_W + 2 * (pp1 % PP_W) + dx;
                f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s = 0; s < 7; s++) {
                    const int k = min(4 * s + lk, 26);
                    const int c = k / 9, r = k - 9 * c;
                    const int ko = c * PL_H * PL_W + (r / 3) * PL_W + (r % 3);
                    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(sA[ab0 + ko], w1[s], c0, 0, 0, 0);
                    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(sA[ab1 + ko], w1[s], c1, 0, 0, 0);
                }
                if (lr < 10) {
#pragma unroll
                    for (int h = 0; h < 2; h++) {
                        if (h == 1 && !two) break;
                        const int pp = (h ? f1 : f0) * 4 + lk;
                        const int py = pp / PP_W, px = pp % PP_W;
                        const int gy = 2 * (oy0 + py), gx = 2 * (ox0 + px);
                        float m = -3.402823466e38f;
                        bool any = false;
#pragma unroll
                        for (int i = 0; i < 4; i++) {
                            bool ok = (gy + (i >> 1) < L1h) && (gx + (i & 1) < L1w);
                            float v = prelu((h ? c1[i] : c0[i]) + b1, a1);
                            if (ok) {
                                m = fmaxf(m, v);
                                any = true;
                            }
                        }
                        // outside the valid pooled map (only feeds discarded cells): keep finite
                        sP[lr * NPP + pp] = any ? m : 0.f;
                    }
                }
            }
        }
        __syncthreads();

        // ---- 3. conv2 (10->16, 3x3) + PReLU on MFMA: M = 18*34 positions (39 frags), N = 16,
        //         K = 90 (+2 zero) in 23 steps; A gathered from the pooled map.
        {
            constexpr int NPOS = PC_H * PC_W;      // 612
            constexpr int NF = (NPOS + 15) / 16;   // 39
            float w2[23];  // per tile (L1-resident): keeps the persistent register set small
#pragma unroll
            for (int s = 0; s < 23; s++) {
                int k = 4 * s + lk;
                w2[s] = k < 90 ? wc.c2w[k * 16 + lr] : 0.f;
            }
            for (int f0 = wave; f0 < ((o.dbg & 4) ? 0 : NF); f0 += 8) {
                const int f1 = f0 + 4;
                const bool two = f1 < NF;
                int p0 = min(f0 * 16 + lr, NPOS - 1), p1 = min((two ? f1 : f0) * 16 + lr, NPOS - 1);
                const int ab0 = (p0 / PC_W) * PP_W + (p0 % PC_W), ab1 = (p1 / PC_W) * PP_W + (p1 % PC_W);
                f32x4 c0 = {0.f, 0.f, 0.f, 0.f}, c1 = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s = 0; s < 23; s++) {
                    const int k = min(4 * s + lk, 89);
                    const int c = k / 9, r = k - 9 * c;
                    const int ko = c * PP_H * PP_W + (r / 3) * PP_W + (r % 3);
                    c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(sP[ab0 + ko], w2[s], c0, 0, 0, 0);
                    c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(sP[ab1 + ko], w2[s], c1, 0, 0, 0);
                }
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    int q0 = f0 * 16 + 4 * lk + i;
                    if (q0 < NPOS) sA[lr * NPOS + q0] = prelu(c0[i] + b2, a2);
                    int q1 = f1 * 16 + 4 * lk + i;
                    if (two && q1 < NPOS) sA[lr * NPOS + q1] = prelu(c1[i] + b2, a2);
                }
            }
        }
        __syncthreads();

        // ---- 4. conv3 (16->32, 3x3) + PReLU on MFMA, computed TRANSPOSED (C = W3^T x im2col:
        //         rows = 32 channels in 2 frags, cols = 16 cells per frag, K = 144 in 36 steps) so
        //         the 1x1 heads are one more MFMA chain summing over the accumulator rows with no
        //         lane movement: Heads^T (16 x cells) = Wh^T (16 x 32) x F (32 x cells), the
        //         k-slot of lane group g at step i being channel 16*mf + 4g + i.
        //         Each wave owns 8 cell fragments (64 accumulator VGPRs); the weights stream
        //         through registers in 4 chunks of 9 k-steps.
        {
            f32x4 acc[8][2];
#pragma unroll
            for (int j = 0; j < 8; j++) acc[j][0] = acc[j][1] = f32x4{0.f, 0.f, 0.f, 0.f};
            int ab[8];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const int f = wave * 8 + j;
                ab[j] = (f >> 1) * PC_W + (f & 1) * 16 + lr;
            }
            const int nchunk = (o.dbg & 8) ? 0 : 4;
            for (int sc = 0; sc < nchunk; sc++) {
                float w3[9][2];
#pragma unroll
                for (int t = 0; t < 9; t++) {
                    const int k = 4 * (9 * sc + t) + lk;
                    w3[t][0] = wc.c3w[k * 32 + lr];
                    w3[t][1] = wc.c3w[k * 32 + 16 + lr];
                }
#pragma unroll
                for (int t = 0; t < 9; t++) {
                    const int k = 4 * (9 * sc + t) + lk;
                    const int c = k / 9, r = k - 9 * c;
                    const int ko = c * PC_H * PC_W + (r / 3) * PC_W + (r % 3);
#pragma unroll
                    for (int j = 0; j < 8; j++) {
                        const float bv = sA[ab[j] + ko];
                        acc[j][0] = __builtin_amdgcn_mfma_f32_16x16x4f32(w3[t][0], bv, acc[j][0], 0, 0, 0);
                        acc[j][1] = __builtin_amdgcn_mfma_f32_16x16x4f32(w3[t][1], bv, acc[j][1], 0, 0, 0);
                    }
                }
            }
            // accumulator row (mf, lk, i) = channel 16*mf + 4*lk + i
            float cb3[2][4], ca3[2][4], hwA[2][4];
#pragma unroll
            for (int mf = 0; mf < 2; mf++)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int ch = 16 * mf + 4 * lk + i;
                    cb3[mf][i] = wc.c3b[ch];
                    ca3[mf][i] = wc.p3[ch];
                    // heads as the A operand: row = head lr (0,1 conv4_1; 2..5 conv4_2), k-slot = ch
                    const int hrow = lr < 2 ? lr * 32 + ch : (lr < 6 ? (lr - 2) * 32 + ch : 0);
                    const float hv = lr < 2 ? wc.c41w[hrow] : wc.c42w[hrow];
                    hwA[mf][i] = lr < 6 ? hv : 0.f;
                }
            const float hb0 = wc.c41b[0], hb1 = wc.c41b[1], hb2 = wc.c42b[0], hb3 = wc.c42b[1];
            const float hb4 = wc.c42b[2], hb5 = wc.c42b[3];
#pragma unroll
            for (int j = 0; j < 8; j++) {
                const int f = wave * 8 + j;
                f32x4 hacc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const float fa = prelu(acc[j][0][i] + cb3[0][i], ca3[0][i]);
                    const float fb = prelu(acc[j][1][i] + cb3[1][i], ca3[1][i]);
                    hacc = __builtin_amdgcn_mfma_f32_16x16x4f32(hwA[0][i], fa, hacc, 0, 0, 0);
                    hacc = __builtin_amdgcn_mfma_f32_16x16x4f32(hwA[1][i], fb, hacc, 0, 0, 0);
                }
                // hacc: lane (cell lr, heads 4*lk + i): group 0 = (a0, a1, r0, r1), group 1 = (r2, r3, -, -)
                const float r2 = __shfl_down(hacc[0], 16), r3 = __shfl_down(hacc[1], 16);
                const int y = f >> 1, x = (f & 1) * 16 + lr;
                const int oy = oy0 + y, ox = ox0 + x;
                const bool valid = (lk == 0) && (oy < P.ph) && (ox < P.pw);
                const float a0 = hacc[0] + hb0, a1v = hacc[1] + hb1;
                const float mx = fmaxf(a0, a1v);
                const float e0 = expf(a0 - mx), e1 = expf(a1v - mx);
                const float prob = __fdiv_rn(e1, e0 + e1);
                const float q0 = hacc[2] + hb2, q1 = hacc[3] + hb3, q2 = r2 + hb4, q3 = r3 + hb5;
                if (DENSE) {
                    if (valid) {
                        int64_t plane = (int64_t)P.ph * P.pw;
                        int64_t cell = (int64_t)oy * P.pw + ox;
                        o.prob[(int64_t)b * plane + cell] = prob;
                        float* rg = o.reg + (int64_t)b * 4 * plane + cell;
                        rg[0] = q0;
                        rg[plane] = q1;
                        rg[2 * plane] = q2;
                        rg[3 * plane] = q3;
                    }
                } else {
                    // mask = prob >= 0.6 (mtcnn.py:183; the python scalar compares as fp32)
                    bool pass = valid && (prob >= 0.6f) && !(o.dbg & 16);
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
            }
        }
        __syncthreads();  // sA/sP are rewritten by the next tile
    }
}

void launch_pnet(bool dense, const uint8_t* frames, int64_t frame_stride, int64_t row_stride, int H, int W,
                 const PNetLevel* d_levels, int n_levels, int64_t total_tiles, const PNetW& w, const PNetOut& o,
                 uint32_t* d_tile_ctr, hipStream_t st) {
    if (total_tiles <= 0) return;
    VTF_HIP(hipMemsetAsync(d_tile_ctr, 0, 4, st));
    int dev = 0, cus = 256;
    VTF_HIP(hipGetDevice(&dev));
    VTF_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    int64_t grid = std::min<int64_t>(total_tiles, (int64_t)cus * PNET_GROUPS_PER_CU);
    if (dense)
        k_pnet<true><<<(unsigned)grid, 256, 0, st>>>(frames, frame_stride, row_stride, H, W, d_levels, n_levels,
                                                      total_tiles, d_tile_ctr, w, o);
    else
        k_pnet<false><<<(unsigned)grid, 256, 0, st>>>(frames, frame_stride, row_stride, H, W, d_levels, n_levels,
                                                       total_tiles, d_tile_ctr, w, o);
}

// ----------------------------------------------------------------------------------- RNet

// LDS plan (floats): A 13552 = conv1 [28][22][22]; later conv2 [48][9][9] @0, pool2 [48][4][4]
// @3888, flat [576] @4656, dense4 [128] @5232.  B 3388 = pool1 [28][11][11].  C 1728 = input.
template <bool FROM_FRAMES>
__global__ __launch_bounds__(256) void k_rnet(const uint8_t* __restrict__ frames, int64_t frame_stride,
                                              int64_t row_stride, int H, int W, const float4* __restrict__ boxes,
                                              const int32_t* __restrict__ img, const float* __restrict__ xin,
                                              RNetW wg, float4* __restrict__ reg_out, float* __restrict__ prob_out,
                                              int32_t* __restrict__ err) {
    const auto wc = to_const(wg);
    __shared__ float sA[13552];
    __shared__ float sB[3388];
    __shared__ float sC[1728];
    const int tid = threadIdx.x;
    const int64_t n = blockIdx.x;
    if (FROM_FRAMES) {
        int y0, x0, hc, wc;
        if (!crop_rect(boxes[n], H, W, y0, x0, hc, wc)) {
            if (tid == 0) atomicAdd(err, 1);
            return;
        }
        const uint8_t* fr = frames + (int64_t)img[n] * frame_stride;
        for (int i = tid; i < 1728; i += 256) {
            int c = i / 576, r = (i / 24) % 24, q = i % 24;
            sC[i] = crop_value(fr, row_stride, c, r, q, y0, x0, hc, wc, 24);
        }
    } else {
        for (int i = tid; i < 1728; i += 256) sC[i] = xin[n * 1728 + i];
    }
    __syncthreads();
    // conv1 3->28 3x3: 22x22
    for (int i = tid; i < 484; i += 256) {
        int y = i / 22, x = i % 22;
        float acc[28];
#pragma unroll
        for (int co = 0; co < 28; co++) acc[co] = wc.c1b[co];
#pragma unroll
        for (int c = 0; c < 3; c++)
#pragma unroll
            for (int ky = 0; ky < 3; ky++)
#pragma unroll
                for (int kx = 0; kx < 3; kx++) {
                    float v = sC[(c * 24 + y + ky) * 24 + x + kx];
                    const VTF_CONST float* wp = wc.c1w + ((c * 3 + ky) * 3 + kx) * 28;
#pragma unroll
                    for (int co = 0; co < 28; co++) acc[co] = fmaf(v, wp[co], acc[co]);
                }
#pragma unroll
        for (int co = 0; co < 28; co++) sA[co * 484 + i] = prelu(acc[co], wc.p1[co]);
    }
    __syncthreads();
    // maxpool 3/2 ceil: 22 -> 11
    for (int i = tid; i < 3388; i += 256) {
        int c = i / 121, y = (i / 11) % 11, x = i % 11;
        float m = -3.402823466e38f;
        for (int dy = 0; dy < 3; dy++)
            for (int dx = 0; dx < 3; dx++) {
                int yy = 2 * y + dy, xx = 2 * x + dx;
                if (yy < 22 && xx < 22) m = fmaxf(m, sA[c * 484 + yy * 22 + xx]);
            }
        sB[i] = m;
    }
    __syncthreads();
    // conv2 28->48 3x3: 9x9; item = (pos, 16-channel group)
    for (int i = tid; i < 81 * 3; i += 256) {
        int pos = i % 81, g = i / 81;
        int y = pos / 9, x = pos % 9;
        float acc[16];
#pragma unroll
        for (int k = 0; k < 16; k++) acc[k] = wc.c2b[g * 16 + k];
        for (int c = 0; c < 28; c++) {
#pragma unroll
            for (int ky = 0; ky < 3; ky++)
#pragma unroll
                for (int kx = 0; kx < 3; kx++) {
                    float v = sB[c * 121 + (y + ky) * 11 + x + kx];
                    const VTF_CONST float* wp = wc.c2w + ((c * 3 + ky) * 3 + kx) * 48 + g * 16;
#pragma unroll
                    for (int k = 0; k < 16; k++) acc[k] = fmaf(v, wp[k], acc[k]);
                }
        }
#pragma unroll
        for (int k = 0; k < 16; k++) sA[(g * 16 + k) * 81 + pos] = prelu(acc[k], wc.p2[g * 16 + k]);
    }
    __syncthreads();
    // maxpool 3/2 ceil: 9 -> 4
    for (int i = tid; i < 768; i += 256) {
        int c = i / 16, y = (i / 4) % 4, x = i % 4;
        float m = -3.402823466e38f;
        for (int dy = 0; dy < 3; dy++)
            for (int dx = 0; dx < 3; dx++) {
                int yy = 2 * y + dy, xx = 2 * x + dx;
                if (yy < 9 && xx < 9) m = fmaxf(m, sA[c * 81 + yy * 9 + xx]);
            }
        sA[3888 + i] = m;
    }
    __syncthreads();
    // conv3 48->64 2x2: 3x3 -> flat (permute 0,3,2,1: index = x*192 + y*64 + c)
    for (int i = tid; i < 9 * 8; i += 256) {
        int pos = i % 9, g = i / 9;
        int y = pos / 3, x = pos % 3;
        float acc[8];
#pragma unroll
        for (int k = 0; k < 8; k++) acc[k] = wc.c3b[g * 8 + k];
        for (int c = 0; c < 48; c++) {
#pragma unroll
            for (int ky = 0; ky < 2; ky++)
#pragma unroll
                for (int kx = 0; kx < 2; kx++) {
                    float v = sA[3888 + c * 16 + (y + ky) * 4 + x + kx];
                    const VTF_CONST float* wp = wc.c3w + ((c * 2 + ky) * 2 + kx) * 64 + g * 8;
#pragma unroll
                    for (int k = 0; k < 8; k++) acc[k] = fmaf(v, wp[k], acc[k]);
                }
        }
#pragma unroll
        for (int k = 0; k < 8; k++) sA[4656 + x * 192 + y * 64 + g * 8 + k] = prelu(acc[k], wc.p3[g * 8 + k]);
    }
    __syncthreads();
    // dense4 576->128 + PReLU; weights transposed [k][128]
    if (tid < 128) {
        float acc = wc.d4b[tid];
        for (int k = 0; k < 576; k++) acc = fmaf(sA[4656 + k], wc.d4w[k * 128 + tid], acc);
        sA[5232 + tid] = prelu(acc, wc.p4[tid]);
    }
    __syncthreads();
    if (tid < 64) {
        // heads: dense5_1 (2) softmax, dense5_2 (4); wave reduction over 128 inputs
        float part[6];
#pragma unroll
        for (int j = 0; j < 6; j++) part[j] = 0.f;
        for (int k = tid; k < 128; k += 64) {
            float f = sA[5232 + k];
            part[0] = fmaf(f, wc.d51w[k], part[0]);
            part[1] = fmaf(f, wc.d51w[128 + k], part[1]);
#pragma unroll
            for (int j = 0; j < 4; j++) part[2 + j] = fmaf(f, wc.d52w[j * 128 + k], part[2 + j]);
        }
#pragma unroll
        for (int j = 0; j < 6; j++)
            for (int off = 32; off > 0; off >>= 1) part[j] += __shfl_xor(part[j], off);
        if (tid == 0) {
            float a0 = part[0] + wc.d51b[0], a1 = part[1] + wc.d51b[1];
            float mx = fmaxf(a0, a1);
            float e0 = expf(a0 - mx), e1 = expf(a1 - mx);
            prob_out[n] = e1 * __fdiv_rn(1.0f, e0 + e1);
            reg_out[n] = make_float4(part[2] + wc.d52b[0], part[3] + wc.d52b[1], part[4] + wc.d52b[2], part[5] + wc.d52b[3]);
        }
    }
}

void launch_rnet(const uint8_t* frames, int64_t frame_stride, int64_t row_stride, int H, int W, const float4* boxes,
                 const int32_t* img, const float* xin, int64_t n, const RNetW& w, float4* reg, float* prob,
                 int32_t* err, hipStream_t st) {
    if (n <= 0) return;
    if (xin)
        k_rnet<false><<<(unsigned)n, 256, 0, st>>>(frames, frame_stride, row_stride, H, W, boxes, img, xin, w, reg,
                                                    prob, err);
    else
        k_rnet<true><<<(unsigned)n, 256, 0, st>>>(frames, frame_stride, row_stride, H, W, boxes, img, xin, w, reg,
                                                   prob, err);
}

// ----------------------------------------------------------------------------------- ONet

// LDS plan (floats): X 14112 = input [3][48][48] (6912) / conv2 half [32][21][21] (14112) /
// later conv3 [64][8][8] @0 (4096), pool3 [64][4][4] @4096 (1024), conv4 flat [1152] @5120,
// dense5 [256] @6272.  Y 16928 = pool1 [32][23][23].  Z 6400 = pool2 [64][10][10].
template <bool FROM_FRAMES>
__global__ __launch_bounds__(512) void k_onet(const uint8_t* __restrict__ frames, int64_t frame_stride,
                                              int64_t row_stride, int H, int W, const float4* __restrict__ boxes,
                                              const int32_t* __restrict__ img, const float* __restrict__ xin,
                                              ONetW wg, float4* __restrict__ reg_out, float* __restrict__ lm_out,
                                              float* __restrict__ prob_out, int32_t* __restrict__ err) {
    const auto wc = to_const(wg);
    __shared__ float sX[14112];
    __shared__ float sY[16928];
    __shared__ float sZ[6400];
    const int tid = threadIdx.x;
    const int64_t n = blockIdx.x;
    if (FROM_FRAMES) {
        int y0, x0, hc, wc;
        if (!crop_rect(boxes[n], H, W, y0, x0, hc, wc)) {
            if (tid == 0) atomicAdd(err, 1);
            return;
        }
        const uint8_t* fr = frames + (int64_t)img[n] * frame_stride;
        for (int i = tid; i < 6912; i += 512) {
            int c = i / 2304, r = (i / 48) % 48, q = i % 48;
            sX[i] = crop_value(fr, row_stride, c, r, q, y0, x0, hc, wc, 48);
        }
    } else {
        for (int i = tid; i < 6912; i += 512) sX[i] = xin[n * 6912 + i];
    }
    __syncthreads();
    // conv1 3->32 3x3 (46x46) + PReLU + maxpool 3/2 ceil (23x23), fused: each item is one
    // pooled position; its <= 3x3 conv1 window is recomputed (conv1 is cheap: K=27).
    for (int i = tid; i < 529; i += 512) {
        int py = i / 23, px = i % 23;
        float m[32];
#pragma unroll
        for (int co = 0; co < 32; co++) m[co] = -3.402823466e38f;
        for (int dy = 0; dy < 3; dy++) {
            int y = 2 * py + dy;
            if (y >= 46) break;
            for (int dx = 0; dx < 3; dx++) {
                int x = 2 * px + dx;
                if (x >= 46) break;
                float acc[32];
#pragma unroll
                for (int co = 0; co < 32; co++) acc[co] = wc.c1b[co];
#pragma unroll
                for (int c = 0; c < 3; c++)
#pragma unroll
                    for (int ky = 0; ky < 3; ky++)
#pragma unroll
                        for (int kx = 0; kx < 3; kx++) {
                            float v = sX[(c * 48 + y + ky) * 48 + x + kx];
                            const VTF_CONST float* wp = wc.c1w + ((c * 3 + ky) * 3 + kx) * 32;
#pragma unroll
                            for (int co = 0; co < 32; co++) acc[co] = fmaf(v, wp[co], acc[co]);
                        }
#pragma unroll
                for (int co = 0; co < 32; co++) m[co] = fmaxf(m[co], prelu(acc[co], wc.p1[co]));
            }
        }
#pragma unroll
        for (int co = 0; co < 32; co++) sY[co * 529 + i] = m[co];
    }
    __syncthreads();
    // conv2 32->64 3x3 (21x21) in two halves of 32 channels, each + PReLU + maxpool 3/2 ceil (10x10)
    for (int half = 0; half < 2; half++) {
        for (int i = tid; i < 441 * 4; i += 512) {
            int pos = i % 441, g = i / 441;  // 8-channel group within the half
            int y = pos / 21, x = pos % 21;
            int cb = half * 32 + g * 8;
            float acc[8];
#pragma unroll
            for (int k = 0; k < 8; k++) acc[k] = wc.c2b[cb + k];
            for (int c = 0; c < 32; c++) {
#pragma unroll
                for (int ky = 0; ky < 3; ky++)
#pragma unroll
                    for (int kx = 0; kx < 3; kx++) {
                        float v = sY[c * 529 + (y + ky) * 23 + x + kx];
                        const VTF_CONST float* wp = wc.c2w + ((c * 3 + ky) * 3 + kx) * 64 + cb;
#pragma unroll
                        for (int k = 0; k < 8; k++) acc[k] = fmaf(v, wp[k], acc[k]);
                    }
            }
#pragma unroll
            for (int k = 0; k < 8; k++) sX[(g * 8 + k) * 441 + pos] = prelu(acc[k], wc.p2[cb + k]);
        }
        __syncthreads();
        for (int i = tid; i < 3200; i += 512) {
            int c = i / 100, y = (i / 10) % 10, x = i % 10;
            float m = -3.402823466e38f;
            for (int dy = 0; dy < 3; dy++)
                for (int dx = 0; dx < 3; dx++) {
                    int yy = 2 * y + dy, xx = 2 * x + dx;
                    if (yy < 21 && xx < 21) m = fmaxf(m, sX[c * 441 + yy * 21 + xx]);
                }
            sZ[(half * 32 + c) * 100 + y * 10 + x] = m;
        }
        __syncthreads();
    }
    // conv3 64->64 3x3 (8x8) + PReLU
    for (int i = tid; i < 64 * 8; i += 512) {
        int pos = i % 64, g = i / 64;
        int y = pos / 8, x = pos % 8;
        float acc[8];
#pragma unroll
        for (int k = 0; k < 8; k++) acc[k] = wc.c3b[g * 8 + k];
        for (int c = 0; c < 64; c++) {
#pragma unroll
            for (int ky = 0; ky < 3; ky++)
#pragma unroll
                for (int kx = 0; kx < 3; kx++) {
                    float v = sZ[c * 100 + (y + ky) * 10 + x + kx];
                    const VTF_CONST float* wp = wc.c3w + ((c * 3 + ky) * 3 + kx) * 64 + g * 8;
#pragma unroll
                    for (int k = 0; k < 8; k++) acc[k] = fmaf(v, wp[k], acc[k]);
                }
        }
#pragma unroll
        for (int k = 0; k < 8; k++) sX[(g * 8 + k) * 64 + pos] = prelu(acc[k], wc.p3[g * 8 + k]);
    }
    __syncthreads();
    // maxpool 2/2 ceil: 8 -> 4
    for (int i = tid; i < 1024; i += 512) {
        int c = i / 16, y = (i / 4) % 4, x = i % 4;
        float m = -3.402823466e38f;
        for (int dy = 0; dy < 2; dy++)
            for (int dx = 0; dx < 2; dx++) m = fmaxf(m, sX[c * 64 + (2 * y + dy) * 8 + 2 * x + dx]);
        sX[4096 + i] = m;
    }
    __syncthreads();
    // conv4 64->128 2x2 (3x3) + PReLU -> flat (x*384 + y*128 + c)
    for (int i = tid; i < 9 * 16; i += 512) {
        int pos = i % 9, g = i / 9;
        int y = pos / 3, x = pos % 3;
        float acc[8];
#pragma unroll
        for (int k = 0; k < 8; k++) acc[k] = wc.c4b[g * 8 + k];
        for (int c = 0; c < 64; c++) {
#pragma unroll
            for (int ky = 0; ky < 2; ky++)
#pragma unroll
                for (int kx = 0; kx < 2; kx++) {
                    float v = sX[4096 + c * 16 + (y + ky) * 4 + x + kx];
                    const VTF_CONST float* wp = wc.c4w + ((c * 2 + ky) * 2 + kx) * 128 + g * 8;
#pragma unroll
                    for (int k = 0; k < 8; k++) acc[k] = fmaf(v, wp[k], acc[k]);
                }
        }
#pragma unroll
        for (int k = 0; k < 8; k++) sX[5120 + x * 384 + y * 128 + g * 8 + k] = prelu(acc[k], wc.p4[g * 8 + k]);
    }
    __syncthreads();
    // dense5 1152->256 + PReLU (weights transposed [k][256])
    if (tid < 256) {
        float acc = wc.d5b[tid];
        for (int k = 0; k < 1152; k++) acc = fmaf(sX[5120 + k], wc.d5w[k * 256 + tid], acc);
        sX[6272 + tid] = prelu(acc, wc.p5[tid]);
    }
    __syncthreads();
    if (tid < 64) {
        float part[16];
#pragma unroll
        for (int j = 0; j < 16; j++) part[j] = 0.f;
        for (int k = tid; k < 256; k += 64) {
            float f = sX[6272 + k];
            part[0] = fmaf(f, wc.d61w[k], part[0]);
            part[1] = fmaf(f, wc.d61w[256 + k], part[1]);
#pragma unroll
            for (int j = 0; j < 4; j++) part[2 + j] = fmaf(f, wc.d62w[j * 256 + k], part[2 + j]);
#pragma unroll
            for (int j = 0; j < 10; j++) part[6 + j] = fmaf(f, wc.d63w[j * 256 + k], part[6 + j]);
        }
#pragma unroll
        for (int j = 0; j < 16; j++)
            for (int off = 32; off > 0; off >>= 1) part[j] += __shfl_xor(part[j], off);
        if (tid == 0) {
            float a0 = part[0] + wc.d61b[0], a1 = part[1] + wc.d61b[1];
            float mx = fmaxf(a0, a1);
            float e0 = expf(a0 - mx), e1 = expf(a1 - mx);
            prob_out[n] = e1 * __fdiv_rn(1.0f, e0 + e1);
            reg_out[n] = make_float4(part[2] + wc.d62b[0], part[3] + wc.d62b[1], part[4] + wc.d62b[2], part[5] + wc.d62b[3]);
#pragma unroll
            for (int j = 0; j < 10; j++) lm_out[n * 10 + j] = part[6 + j] + wc.d63b[j];
        }
    }
}

void launch_onet(const uint8_t* frames, int64_t frame_stride, int64_t row_stride, int H, int W, const float4* boxes,
                 const int32_t* img, const float* xin, int64_t n, const ONetW& w, float4* reg, float* lm, float* prob,
                 int32_t* err, hipStream_t st) {
    if (n <= 0) return;
    if (xin)
        k_onet<false><<<(unsigned)n, 512, 0, st>>>(frames, frame_stride, row_stride, H, W, boxes, img, xin, w, reg, lm,
                                                    prob, err);
    else
        k_onet<true><<<(unsigned)n, 512, 0, st>>>(frames, frame_stride, row_stride, H, W, boxes, img, xin, w, reg, lm,
                                                   prob, err);
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
                                int32_t* __restrict__ iout) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
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
                               int32_t* __restrict__ out) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < n && flag[k]) out[incl[k] - 1] = (int32_t)k;
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
__global__ void k_iom_chain(const float4* __restrict__ boxes, const int32_t* __restrict__ img,
                            const int32_t* __restrict__ order, int64_t n, float thr, int32_t* __restrict__ keep) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= n) return;
    int32_t j = order[k];
    float4 b2 = boxes[j];
    int32_t ij = img[j];
    int drop = 0;
    for (int64_t q = 0; q < k && !drop; q++) {
        int32_t i = order[q];
        if (img[i] != ij) continue;
        float4 b1 = boxes[i];
        float iw = (fminf(b1.z, b2.z) - fmaxf(b1.x, b2.x)) + 1.0f;
        float ih = (fminf(b1.w, b2.w) - fmaxf(b1.y, b2.y)) + 1.0f;
        if (!(iw > 0.f && ih > 0.f)) continue;
        float inter = iw * ih;
        float a1 = ((b1.z - b1.x) + 1.0f) * ((b1.w - b1.y) + 1.0f);
        float a2 = ((b2.z - b2.x) + 1.0f) * ((b2.w - b2.y) + 1.0f);
        float iom = __fdiv_rn(inter, fminf(a1, a2));
        if (iom > thr) drop = 1;
    }
    keep[k] = !drop;
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
                          float4* rout, int32_t* iout, hipStream_t st) {
    if (n > 0)
        k_gather_refine<<<cdiv(n, 256), 256, 0, st>>>(idx, n, bin, sin, rin, iin, refine, plus_one, square, bout, sout,
                                                       rout, iout);
}
void launch_threshold(const float* s, int64_t n, float thr, int32_t* flag, hipStream_t st) {
    if (n > 0) k_threshold<<<cdiv(n, 256), 256, 0, st>>>(s, n, thr, flag);
}
void launch_flag_compact(const int32_t* flag, const int32_t* incl, int64_t n, int32_t* out, hipStream_t st) {
    if (n > 0) k_flag_compact<<<cdiv(n, 256), 256, 0, st>>>(flag, incl, n, out);
}
void launch_landmarks(const float4* boxes, const float* lm, int64_t n, float* out, hipStream_t st) {
    if (n > 0) k_landmarks<<<cdiv(n, 256), 256, 0, st>>>(boxes, lm, n, out);
}
void launch_iom_chain(const float4* boxes, const int32_t* img, const int32_t* order, int64_t n, float thr,
                      int32_t* keep, hipStream_t st) {
    if (n > 0) k_iom_chain<<<cdiv(n, 128), 128, 0, st>>>(boxes, img, order, n, thr, keep);
}

}  // namespace vtf

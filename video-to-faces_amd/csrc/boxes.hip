// Box post-processing on device: the reference's host loop over detector boxes
// (detection.py:126-145 process_frames_batch steps 2-5) as one kernel, so face crops go from the
// detector's device rows to the encoder's blob kernel without a host round trip.
//
//   filter_boxes (detection.py:174-180) + check_box (165-171):
//     (floor x1, floor y1, ceil x2, ceil y2) of the fp32 box; reject when
//     score < min_score, width or height < min_size, or (min_border != 0) the box is closer than
//     min_border to a frame edge.  The score compare is fp32 against fp32(min_score): the
//     reference compares a numpy float32 with a Python float, which NumPy >= 2 (NEP 50, the
//     NumPy this build and its golden vectors run) evaluates in float32.
//   adjust_boxes (detection.py:220-262), unless p.adjust == 0 (filter_boxes alone):
//     scale about the centre in double precision (Python float math) with floor/ceil and the
//     frame clamp, then the integer squaring with its out-of-frame shift and the final shrink
//     when a side exceeds the other frame dimension.
//
// A det-batch carries at most a few thousand rows (YOLO/R-CNN keep <= 100 per frame), so one
// 1024-thread workgroup walks them in order: a block scan of the keep flags gives each crop its
// output slot, which keeps the reference's (frame, face) order.  Latency-bound by design (a few
// microseconds); it exists to remove the host round trip, not for bandwidth.
#include <algorithm>

#include "boxes.hpp"

namespace vtf {

namespace {

constexpr int BOX_THREADS = 1024;
constexpr int BOX_WAVES = BOX_THREADS / 64;

// exclusive block scan of v; *total = block sum (all threads)
__device__ int block_scan_excl(int v, int* s_wave, int* total) {
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o, 64);
        if (lane >= o) x += y;
    }
    if (lane == 63) s_wave[w] = x;
    __syncthreads();
    if (threadIdx.x == 0) {
        int acc = 0;
        for (int i = 0; i < BOX_WAVES; i++) {
            const int t = s_wave[i];
            s_wave[i] = acc;
            acc += t;
        }
        s_wave[BOX_WAVES] = acc;
    }
    __syncthreads();
    const int r = x - v + s_wave[w];
    *total = s_wave[BOX_WAVES];
    __syncthreads();
    return r;
}

// one side of the squaring step: widen [a1, a2) by d inside [0, lim], shifting back in when a
// side leaves the frame
__device__ inline void widen(int& a1, int& a2, int d, int lim) {
    a1 -= d / 2;
    a2 += d - d / 2;
    if (a1 < 0) {
        a2 -= a1;
        a1 = 0;
        a2 = min(lim, a2);
    }
    if (a2 > lim) {
        a1 -= a2 - lim;
        a2 = lim;
        a1 = max(0, a1);
    }
}

__device__ inline void narrow(int& a1, int& a2, int d) {
    a1 += d / 2;
    a2 -= d - d / 2;
}

// scale one axis about the centre: [floor(max(0, c - s_lo*len/2)), ceil(min(lim, c + s_hi*len/2))]
__device__ inline void scale_axis(int& a1, int& a2, double s_lo, double s_hi, int lim) {
    const int len = a2 - a1;
    const double c = (double)a1 + (double)len / 2.0;
    const double lo = c - s_lo * (double)len / 2.0;
    const double hi = c + s_hi * (double)len / 2.0;
    a1 = (int)floor(lo < 0.0 ? 0.0 : lo);
    a2 = (int)ceil((double)lim < hi ? (double)lim : hi);
}

__global__ __launch_bounds__(BOX_THREADS) void k_box_post(const float* __restrict__ rows,
                                                          const int32_t* __restrict__ counts, int B, int H, int W,
                                                          vtf_box_params p, int frame_offset,
                                                          int32_t* __restrict__ crops, int32_t* __restrict__ src,
                                                          int32_t* __restrict__ frame_counts,
                                                          int32_t* __restrict__ total_out, int64_t cap) {
    __shared__ int s_beg[BOX_MAX_FRAMES + 1];
    __shared__ int s_kept[BOX_MAX_FRAMES];
    __shared__ int s_wave[BOX_WAVES + 1];
    const int tid = threadIdx.x;
    // exclusive prefix of the per-frame row counts
    const int per = (B + BOX_THREADS - 1) / BOX_THREADS;
    int part = 0;
    for (int j = 0; j < per; j++) {
        const int f = tid * per + j;
        if (f < B) part += max(0, counts[f]);
    }
    int n = 0;
    int acc = block_scan_excl(part, s_wave, &n);
    for (int j = 0; j < per; j++) {
        const int f = tid * per + j;
        if (f < B) {
            s_beg[f] = acc;
            s_kept[f] = 0;
            acc += max(0, counts[f]);
        }
    }
    if (tid == 0) s_beg[B] = n;
    __syncthreads();
    const float min_score = p.min_score;
    int base = 0;
    for (int c0 = 0; c0 < n; c0 += BOX_THREADS) {
        const int i = c0 + tid;
        int keep = 0, f = 0, x1 = 0, y1 = 0, x2 = 0, y2 = 0;
        if (i < n) {
            int lo = 0, hi = B;
            while (hi - lo > 1) {
                const int mid = (lo + hi) >> 1;
                if (s_beg[mid] <= i) lo = mid; else hi = mid;
            }
            f = lo;
            const float* r = rows + (int64_t)i * 5;
            x1 = (int)floorf(r[0]);
            y1 = (int)floorf(r[1]);
            x2 = (int)ceilf(r[2]);
            y2 = (int)ceilf(r[3]);
            const bool low = r[4] < min_score;
            const bool small = (double)(x2 - x1) < p.min_size || (double)(y2 - y1) < p.min_size;
            const double mb = p.min_border;
            const bool edge = mb != 0.0 && ((double)x1 < mb || (double)y1 < mb || (double)x2 > (double)W - mb ||
                                            (double)y2 > (double)H - mb);
            keep = !(low || small || edge);
            if (keep && p.adjust) {
                scale_axis(x1, x2, p.scale[0], p.scale[1], W);
                scale_axis(y1, y2, p.scale[2], p.scale[3], H);
                if (p.square) {
                    const int w = x2 - x1, h = y2 - y1;
                    if (h > w)
                        widen(x1, x2, h - w, W);
                    else if (w > h)
                        widen(y1, y2, w - h, H);
                    const int w2 = x2 - x1, h2 = y2 - y1;
                    if (w2 > H)
                        narrow(x1, x2, w2 - H);
                    else if (h2 > W)
                        narrow(y1, y2, h2 - W);
                }
            }
        }
        int nk = 0;
        const int pos = block_scan_excl(keep, s_wave, &nk);
        if (keep && base + pos < cap) {  // (past cap: counted, not written; the host reports it)
            int32_t* o = crops + (int64_t)(base + pos) * 5;
            o[0] = frame_offset + f;
            o[1] = x1;
            o[2] = y1;
            o[3] = x2;
            o[4] = y2;
            if (src) src[base + pos] = i;
            atomicAdd(&s_kept[f], 1);
        }
        base += nk;
    }
    __syncthreads();
    for (int f = tid; f < B; f += BOX_THREADS) frame_counts[f] = s_kept[f];
    if (tid == 0) *total_out = base;
}

}  // namespace

void launch_box_post(const float* d_rows, const int32_t* d_counts, int B, int H, int W, const vtf_box_params& p,
                     int frame_offset, int32_t* d_crops, int32_t* d_src, int32_t* d_frame_counts, int32_t* d_total,
                     hipStream_t st, int64_t cap) {
    VTF_CHECK(B > 0 && B <= BOX_MAX_FRAMES, VTF_E_LIMIT, "box post-processing: 1..4096 frames per call");
    k_box_post<<<1, BOX_THREADS, 0, st>>>(d_rows, d_counts, B, H, W, p, frame_offset, d_crops, d_src, d_frame_counts,
                                          d_total, cap);
    VTF_HIP(hipGetLastError());
}

int64_t rows_to_crops(Arena& ar, int slot, const float* d_rows, const std::vector<int32_t>& counts, int H, int W,
                      const vtf_box_params& p, int frame_offset, int32_t* d_crops, int32_t* d_src,
                      int32_t* h_frame_counts, int64_t cap, int64_t* out_n, hipStream_t st) {
    const int B = (int)counts.size();
    int64_t rows = 0;
    for (int32_t c : counts) rows += std::max(0, c);
    if (out_n) *out_n = rows;
    VTF_CHECK(rows <= cap, VTF_E_CAPACITY, "crop capacity too small (bound: detector rows)");
    // pinned mailbox (Arena::mail): [0, B) counts in, [B, 2B) kept per frame, [2B] total -- the
    // kernel reads the counts and writes its results there directly (no blit copies, no memset)
    Arena::Mail mb = ar.mail(slot, (2 * (size_t)B + 1) * 4);
    int32_t* h = (int32_t*)mb.h;
    int32_t* d = (int32_t*)mb.d;
    std::copy(counts.begin(), counts.end(), h);
    if (rows > 0) {
        launch_box_post(d_rows, d, B, H, W, p, frame_offset, d_crops, d_src, d + B, d + 2 * B, st);
        VTF_HIP(hipStreamSynchronize(st));
    } else {
        std::fill(h + B, h + 2 * B + 1, 0);
    }
    if (h_frame_counts) std::copy(h + B, h + 2 * B, h_frame_counts);
    if (out_n) *out_n = h[2 * (size_t)B];
    return h[2 * (size_t)B];
}

void check_crops_host(const int32_t* crops, int64_t N, int F, int H, int W) {
    for (int64_t i = 0; i < N; i++) {
        const int32_t* c = crops + i * 5;
        VTF_CHECK(c[0] >= 0 && c[0] < F, VTF_E_ARG, "crop " + std::to_string(i) + ": frame index out of range");
        VTF_CHECK(c[1] >= 0 && c[1] < c[3] && c[3] <= W && c[2] >= 0 && c[2] < c[4] && c[4] <= H, VTF_E_ARG,
                  "crop " + std::to_string(i) + ": empty or outside the frame (cv2.resize of an empty slice fails)");
    }
}

}  // namespace vtf

using namespace vtf;

extern "C" int vtf_boxes_to_crops(const float* d_rows, const int32_t* counts, int B, int H, int W,
                                  const vtf_box_params* params, int32_t frame_offset, int32_t* d_crops,
                                  int32_t* d_src, int32_t* out_frame_counts, int64_t cap, int64_t* out_n,
                                  void* hip_stream) {
    return guarded_on(stream_device((hipStream_t)hip_stream), [&] {
        VTF_CHECK(counts && params && out_n && B > 0 && H > 0 && W > 0, VTF_E_ARG, "bad argument");
        std::vector<int32_t> c(counts, counts + B);
        int64_t rows = 0;
        for (int32_t v : c) rows += std::max(0, v);
        VTF_CHECK(rows == 0 || (d_rows && d_crops), VTF_E_ARG, "null argument");
        hipStream_t st = (hipStream_t)hip_stream;
        StreamScratch sc = stream_scratch(st);
        rows_to_crops(*sc.ar, 0, d_rows, c, H, W, *params, frame_offset, d_crops, d_src, out_frame_counts, cap, out_n,
                      st);
    });
}

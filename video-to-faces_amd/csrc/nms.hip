// Greedy NMS with torchvision semantics on gfx950.
//
// Replaces torchvision.ops.batched_nms / nms (third-party C++ op; the reference calls it at
// src/videotofaces/detectors/mtcnn.py:196,205,219 and detectors/operations/post.py:8).
// Semantics restated (torchvision/ops/boxes.py, csrc/ops/cpu/nms_kernel.cpp):
//   * n*4 > 4000 -> "vanilla": independent NMS per class id, result sorted by score;
//     else "coordinate trick": boxes += float(idx) * (max(boxes) + 1), one NMS.
//   * NMS: stable descending score order; areas (x2-x1)*(y2-y1) in fp32; keep i unless
//     suppressed; suppress j if inter / ((area_i + area_j) - inter) > thr (fp32 IoU promoted
//     to double).  Output: keep indices ordered by (score desc, index asc).
// Design (MI355X): a stable sort by (call, image, score desc) gives every segment's order;
// an IoU bitmask kernel (one wave per 64-row block x column-block chunk, boxes broadcast through
// LDS) writes u64 suppression words; one workgroup per segment resolves the greedy chain 64 rows
// per step (fixed-point diagonal, one barrier per step) and writes the segment's kept list; one
// last launch merges a vanilla call's image lists into torchvision's output order.
// Build with -ffp-contract=off: every IoU op is rounded exactly like the CPU kernel.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>

#include <algorithm>

#include "common.hpp"
#include "nms.hpp"

namespace vtf {

// nms_multi's first launch.  Block 0 copies the call / segment tables from the host mailbox
// (pinned, mapped) into device memory for the later kernels and zeroes the coordinate-trick base of
// every call without one; block 1 + i computes the box maximum of trick call trick[i] (the
// coordinate-trick offset base, torchvision batched_nms), reading its bounds from the mailbox.
__global__ void k_nms_prep(const uint8_t* __restrict__ mail, uint8_t* __restrict__ tables, int bytes,
                           const float4* __restrict__ boxes, size_t o_cbeg, size_t o_cn, size_t o_van, size_t o_trick,
                           int C, float* __restrict__ call_max, int32_t* __restrict__ ovf_flag,
                           int32_t* __restrict__ seg_ctr, int n_ctr, int32_t* __restrict__ dtie) {
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) *ovf_flag = 0;
        for (int i = threadIdx.x; i < n_ctr; i += blockDim.x) seg_ctr[i] = 0;  // segment counters
        const uint32_t* src = (const uint32_t*)mail;
        uint32_t* dst = (uint32_t*)tables;
        for (int i = threadIdx.x; i < bytes / 4; i += blockDim.x) dst[i] = src[i];
        const int64_t* cn = (const int64_t*)(mail + o_cn);
        const uint8_t* van = mail + o_van;
        for (int c = threadIdx.x; c < C; c += blockDim.x) {
            if (van[c] || cn[c] == 0) call_max[c] = 0.f;
            ovf_flag[1 + c] = 0;  // tie flags
            dtie[c] = 0;          // (device copy)
        }
        return;
    }
    const int c = ((const int32_t*)(mail + o_trick))[blockIdx.x - 1];
    const int64_t beg = ((const int64_t*)(mail + o_cbeg))[c], n = ((const int64_t*)(mail + o_cn))[c];
    // torch's max propagates NaN (boxes.max() in batched_nms): so does this one
    auto nmax = [](float a, float b) { return (a != a || b != b) ? NAN : fmaxf(a, b); };
    float m = -INFINITY;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        float4 b = boxes[beg + i];
        m = nmax(m, nmax(nmax(b.x, b.y), nmax(b.z, b.w)));
    }
    __shared__ float red[256];
    red[threadIdx.x] = m;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] = nmax(red[threadIdx.x], red[threadIdx.x + s]);
        __syncthreads();
    }
    if (threadIdx.x == 0) call_max[c] = red[0];
}

// key = [call][seg image: sbits] [desc score:32], only as many high bits as the call / image
// counts need (the radix sort runs end_bit / 8 passes); element order is position order.
__global__ void k_seg_keys(const float* __restrict__ scores, const int32_t* __restrict__ img,
                           const int32_t* __restrict__ elem_call, const uint8_t* __restrict__ call_vanilla,
                           int64_t N, int with_seg, int sbits, uint64_t* __restrict__ keys, int32_t* __restrict__ vals) {
    int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= N) return;
    uint32_t c = (uint32_t)elem_call[e];
    uint32_t s = (with_seg && call_vanilla[c]) ? (uint32_t)img[e] : 0u;
    keys[e] = ((uint64_t)((c << sbits) | s) << 32) | desc_key(scores[e]);
    vals[e] = (int32_t)e;
}

// lower_bound of (hi << 32) in the sorted keys for every segment id (no atomics: a
// segment's elements are contiguous after the sort)
__global__ void k_seg_bounds(const uint64_t* __restrict__ keys, int64_t N, const uint32_t* __restrict__ seg_hi,
                             int S, int64_t* __restrict__ seg_start) {
    int s = blockIdx.x * blockDim.x + threadIdx.x;
    if (s > S) return;
    if (s == S) {
        seg_start[S] = N;
        return;
    }
    uint64_t target = (uint64_t)seg_hi[s] << 32;
    int64_t lo = 0, hi = N;
    while (lo < hi) {
        int64_t mid = (lo + hi) >> 1;
        if (keys[mid] < target) lo = mid + 1; else hi = mid;
    }
    seg_start[s] = lo;
}

// exclusive prefix of cnt[0, S) into koff[0, S] (LDS) by one block of NT threads (part: NT ints)
template <int NT>
__device__ inline void block_prefix(const int32_t* __restrict__ cnt, int S, int32_t* koff, int32_t* part) {
    const int tid = threadIdx.x;
    const int q = (S + NT - 1) / NT, a0 = min(S, tid * q), a1 = min(S, a0 + q);
    int sum = 0;
    for (int i = a0; i < a1; i++) sum += cnt[i];
    part[tid] = sum;
    __syncthreads();
    if (tid < 64) {  // one wave scans the NT partial sums
        int carry = 0;
        for (int b = 0; b < NT; b += 64) {
            const int v = part[b + tid];
            int x = v;
            for (int o = 1; o < 64; o <<= 1) {
                const int y = __shfl_up(x, o);
                if (tid >= o) x += y;
            }
            part[b + tid] = carry + x - v;
            carry += __shfl(x, 63);
        }
        if (tid == 0) koff[S] = carry;
    }
    __syncthreads();
    sum = part[tid];
    for (int i = a0; i < a1; i++) {
        koff[i] = sum;
        sum += cnt[i];
    }
    __syncthreads();
}

// Segmented sort without a device-wide sort (segments of calls bounded by NMS_SORT_BOUND boxes): count
// per segment, scatter (slot order within a segment is arbitrary: the key carries the element index),
// then one workgroup per segment sorts its (descending-score key, element index) keys -- unique keys,
// so the order equals the stable sort by (segment, score desc) over position order.  The network is
// the ascending-only bitonic form (the first step of each merge compares mirrored pairs), so a
// segment needs no padding: positions >= m act as +inf and are never read or written.  Segments of
// up to NMS_SORT_LDS keys sort in LDS, longer ones in place in global memory (one workgroup, the
// same network; the workgroup's waves share the CU's L1, so a barrier orders their accesses).
constexpr int NMS_SORT_LDS = 4096;      // 32 KB of LDS per workgroup
constexpr int64_t NMS_SORT_BOUND = 65536;  // larger calls take the device-wide merge sort
__device__ inline int seg_of(const int32_t* __restrict__ img, const int32_t* __restrict__ elem_call,
                             const uint8_t* __restrict__ van, const int32_t* __restrict__ sbase, int64_t e) {
    const int c = elem_call[e];
    return sbase[c] + (van[c] ? img[e] : 0);
}
// Per-block LDS histograms keep the global atomics to one per (block, segment): a call's boxes
// mostly share few segments, and per-element atomics on those few addresses serialised (~90 us
// per call).  A wave whose elements all fall in one segment adds them with one LDS atomic.
constexpr int SEG_T = 1024, SEG_HIST = 4096;
__global__ __launch_bounds__(SEG_T) void k_seg_count(const int32_t* __restrict__ img, const int32_t* __restrict__ elem_call,
                                                     const uint8_t* __restrict__ van, const int32_t* __restrict__ sbase,
                                                     int64_t N, int S, int32_t* __restrict__ cnt) {
    __shared__ int32_t h[SEG_HIST];
    const int tid = threadIdx.x, lane = tid & 63;
    const bool lds = S <= SEG_HIST;
    if (lds) {
        for (int i = tid; i < S; i += SEG_T) h[i] = 0;
        __syncthreads();
    }
    const int64_t e = (int64_t)blockIdx.x * SEG_T + tid;
    const bool valid = e < N;
    const int sg = valid ? seg_of(img, elem_call, van, sbase, e) : -1;
    if (!lds) {
        if (valid) atomicAdd(&cnt[sg], 1);
        return;
    }
    const int s0 = __builtin_amdgcn_readfirstlane(sg);
    const uint64_t all = __ballot(valid), same = __ballot(valid && sg == s0);
    if (same == all) {
        if (lane == 0 && all) atomicAdd(&h[s0], (int)__popcll(all));
    } else if (valid) {
        atomicAdd(&h[sg], 1);
    }
    __syncthreads();
    for (int i = tid; i < S; i += SEG_T)
        if (h[i]) atomicAdd(&cnt[i], h[i]);
}
// keys of segment s at [sstart[s], sstart[s + 1]) in any slot order: (desc score key | element)
__global__ __launch_bounds__(SEG_T) void k_seg_scatter(const float* __restrict__ scores, const int32_t* __restrict__ img,
                                                       const int32_t* __restrict__ elem_call,
                                                       const uint8_t* __restrict__ van, const int32_t* __restrict__ sbase,
                                                       int64_t N, int S, const int32_t* __restrict__ cnt,
                                                       int32_t* __restrict__ fill, int64_t* __restrict__ sstart,
                                                       uint64_t* __restrict__ tmp) {
    extern __shared__ int32_t soff[];  // [S + 1], then (S <= SEG_HIST) block counts h[S] and bases hb[S]
    __shared__ int32_t part[SEG_T];
    const int tid = threadIdx.x, lane = tid & 63;
    const bool lds = S <= SEG_HIST;
    int32_t* h = soff + S + 1;
    int32_t* hb = h + S;
    if (lds)
        for (int i = tid; i < S; i += SEG_T) h[i] = 0;
    block_prefix<SEG_T>(cnt, S, soff, part);  // (ends with a barrier)
    if (blockIdx.x == 0)
        for (int i = tid; i <= S; i += SEG_T) sstart[i] = soff[i];
    const int64_t e = (int64_t)blockIdx.x * SEG_T + tid;
    const bool valid = e < N;
    const int sg = valid ? seg_of(img, elem_call, van, sbase, e) : 0;
    const uint64_t key = valid ? ((uint64_t)desc_key(scores[e]) << 32) | (uint32_t)e : 0;
    if (!lds) {
        if (valid) tmp[soff[sg] + atomicAdd(&fill[sg], 1)] = key;
        return;
    }
    // local rank: one LDS atomic per wave when the wave's elements share a segment
    const int s0 = __builtin_amdgcn_readfirstlane(sg);
    const uint64_t all = __ballot(valid), same = __ballot(valid && sg == s0);
    int r;
    if (same == all) {
        int b = 0;
        if (lane == 0 && all) b = atomicAdd(&h[s0], (int)__popcll(all));
        b = __shfl(b, 0);
        r = b + (int)__popcll(all & ((1ull << lane) - 1ull));
    } else {
        r = valid ? atomicAdd(&h[sg], 1) : 0;
    }
    __syncthreads();
    for (int i = tid; i < S; i += SEG_T)
        if (h[i]) hb[i] = atomicAdd(&fill[i], h[i]);
    __syncthreads();
    if (valid) tmp[soff[sg] + hb[sg] + r] = key;
}
// ascending bitonic network over a[0, m) (1024 threads, one workgroup)
template <class P>
__device__ inline void bitonic_asc(P a, int m) {
    const int tid = threadIdx.x;
    int n2 = 1;
    while (n2 < m) n2 <<= 1;
    for (int k = 2; k <= n2; k <<= 1) {
        const int h = k >> 1;
        for (int t = tid; t < n2 / 2; t += 1024) {  // merge step 1: mirrored pairs of each k block
            const int b = t / h, o = t - b * h;
            const int i = b * k + o, l = b * k + k - 1 - o;
            if (l < m) {
                const uint64_t x = a[i], y = a[l];
                if (x > y) a[i] = y, a[l] = x;
            }
        }
        __syncthreads();
        for (int j = h >> 1; j > 0; j >>= 1) {  // half-cleaners
            for (int t = tid; t < n2 / 2; t += 1024) {
                const int i = 2 * t - (t & (j - 1)), l = i + j;
                if (l < m) {
                    const uint64_t x = a[i], y = a[l];
                    if (x > y) a[i] = y, a[l] = x;
                }
            }
            __syncthreads();
        }
    }
}
__global__ __launch_bounds__(1024) void k_seg_sort(const int64_t* __restrict__ sstart, const uint64_t* __restrict__ tmp,
                                                   uint64_t* __restrict__ ck, int32_t* __restrict__ ord) {
    __shared__ uint64_t a[NMS_SORT_LDS];
    const int tid = threadIdx.x;
    const int64_t beg = sstart[blockIdx.x];
    const int m = (int)(sstart[blockIdx.x + 1] - beg);
    if (m == 0) return;
    if (m <= NMS_SORT_LDS) {
        for (int i = tid; i < m; i += 1024) a[i] = tmp[beg + i];
        __syncthreads();
        bitonic_asc(a, m);
        for (int i = tid; i < m; i += 1024) {
            const uint64_t v = a[i];
            ck[beg + i] = v;
            ord[beg + i] = (int32_t)(uint32_t)v;
        }
    } else {
        uint64_t* g = ck + beg;
        for (int i = tid; i < m; i += 1024) g[i] = tmp[beg + i];
        __syncthreads();
        bitonic_asc(g, m);
        for (int i = tid; i < m; i += 1024) ord[beg + i] = (int32_t)(uint32_t)g[i];
    }
}
// the merge-sort path's keys ((call, image) | desc score) -> (desc score, element index)
__global__ void k_composite(const uint64_t* __restrict__ k1, const int32_t* __restrict__ ord, int64_t N,
                            uint64_t* __restrict__ ck) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (p < N) ck[p] = ((uint64_t)(uint32_t)k1[p] << 32) | (uint32_t)ord[p];
}

struct MaskTask {
    int32_t seg;
    int32_t rb;
    int32_t cb0, cb1;  // column blocks [cb0, cb1) of row block rb (long rows are split over waves)
};
constexpr int MASK_CHUNK = 8;  // column blocks per mask task

// mask tasks of a segment of nb row blocks: row block rb takes ceil((nb - rb) / MASK_CHUNK) tasks, so
// the first rb row blocks take ntasks(nb) - ntasks(nb - rb) (sum_{j=1..n} ceil(j / 8) in closed form)
__host__ __device__ inline int64_t ntasks(int64_t n) {
    const int64_t q = n / MASK_CHUNK, r = n % MASK_CHUNK;
    return (q + 1) * (MASK_CHUNK / 2 * q + r);
}

// Segment plan on the device (one workgroup): from the sorted segment starts, each segment's
// count, mask offset (sum of nb^2 * 64 words before it), coordinate-trick base and its mask tasks
// (rb, column-block chunk) -- what the host used to build after a device->host round trip.  Tasks
// are enumerated segment by segment, row block by row block (any order is correct: each task
// writes its own mask words).
constexpr int PLAN_T = 256;  // (1024 threads waited ~0.27 ms for a CU slot beside the other lanes' k_pnet workgroups; c2 unchanged either way)
__global__ __launch_bounds__(PLAN_T) void k_nms_plan(const int64_t* __restrict__ sstart, const uint32_t* __restrict__ seg_hi,
                                                      int sbits, const uint8_t* __restrict__ call_van,
                                                      const float* __restrict__ call_max, int S, int32_t* __restrict__ scnt,
                                                      int64_t* __restrict__ moff, float* __restrict__ offb,
                                                      int64_t* __restrict__ toff, MaskTask* __restrict__ tasks,
                                                      int32_t* __restrict__ n_tasks, int64_t max_tasks) {
    __shared__ int64_t w_m[PLAN_T / 64], w_t[PLAN_T / 64];
    __shared__ int64_t carry_m, carry_t;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    if (tid == 0) carry_m = carry_t = 0;
    __syncthreads();
    // pass 1: counts, exclusive prefix sums of mask words and tasks (chunks of PLAN_T segments)
    for (int s0 = 0; s0 < S; s0 += PLAN_T) {
        const int s = s0 + tid;
        int64_t nm = 0, nt = 0;
        if (s < S) {
            const int64_t m = sstart[s + 1] - sstart[s];
            const int64_t nb = (m + 63) >> 6;
            nm = nb * nb * 64;
            nt = ntasks(nb);
            scnt[s] = (int32_t)m;
            const uint32_t c = seg_hi[s] >> sbits;
            offb[s] = call_van[c] ? 0.f : call_max[c] + 1.0f;
        }
        int64_t im = nm, it = nt;  // inclusive wave scans
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t a = __shfl_up(im, o), b = __shfl_up(it, o);
            if (lane >= o) im += a, it += b;
        }
        if (lane == 63) w_m[wave] = im, w_t[wave] = it;
        __syncthreads();
        int64_t bm = carry_m, bt = carry_t;
        for (int w = 0; w < wave; w++) bm += w_m[w], bt += w_t[w];
        if (s < S) {
            moff[s] = bm + im - nm;
            toff[s] = bt + it - nt;
        }
        __syncthreads();
        if (tid == PLAN_T - 1) carry_m = bm + im, carry_t = bt + it;
        __syncthreads();
    }
    const int64_t T = carry_t;
    if (tid == 0) {
        toff[S] = T;
        *n_tasks = (int32_t)min(T, max_tasks);
    }
    __syncthreads();
    // pass 2: every task, by binary search of its segment and row block
    for (int64_t t = tid; t < min(T, max_tasks); t += PLAN_T) {
        int lo = 0, hi = S - 1;  // last segment with toff <= t
        while (lo < hi) {
            const int mid = (lo + hi + 1) >> 1;
            if (toff[mid] <= t) lo = mid; else hi = mid - 1;
        }
        const int s = lo;
        const int64_t local = t - toff[s];
        const int64_t nb = ((int64_t)scnt[s] + 63) >> 6, all = ntasks(nb);
        int64_t a = 0, b = nb - 1;  // last rb with P(rb) = all - ntasks(nb - rb) <= local
        while (a < b) {
            const int64_t mid = (a + b + 1) >> 1;
            if (all - ntasks(nb - mid) <= local) a = mid; else b = mid - 1;
        }
        const int64_t rb = a, c0 = rb + MASK_CHUNK * (local - (all - ntasks(nb - rb)));
        tasks[t] = MaskTask{s, (int32_t)rb, (int32_t)c0, (int32_t)min(nb, c0 + MASK_CHUNK)};
    }
}

__device__ inline float4 load_box(const float4* __restrict__ boxes, const int32_t* __restrict__ img,
                                  int32_t e, float off_base) {
    float4 b = boxes[e];
    if (off_base != 0.f) {
        float off = (float)img[e] * off_base;
        b.x = b.x + off;
        b.y = b.y + off;
        b.z = b.z + off;
        b.w = b.w + off;
    }
    return b;
}

// IoU test without the division.  The reference suppresses j when (double)fl(inter / uni) > thr
// (torchvision nms_kernel.cpp: float IoU, double threshold).  fl(q) is a float, so that is
// fl(q) >= F, F the smallest float above thr; under round-to-nearest-even fl(q) >= F iff
// q > mid, or q == mid with F's significand even, mid = (F- + F) / 2 the midpoint below F.  For
// uni > 0 that is inter > mid * uni (or >=) in double, where mid (25 bits) times uni (24 bits)
// and inter are exact: the same decision bit for bit.  uni <= 0 or NaN (degenerate boxes) take
// the IEEE division, as the reference does.
struct IouThr {
    double thr, mid;
    int ge;  // F's significand is even: q == mid suppresses
};

// One wave per (segment, 64-row block, chunk of column blocks >= rb): lane = row, the 64 column
// boxes of a block are broadcast from LDS and all 64 tested unrolled (branch-free; the diagonal
// block's lower triangle and columns past the segment are masked afterwards).
__device__ inline float vmax(float a, float b) {
    float r;
    asm("v_max_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}
__device__ inline float vmin(float a, float b) {
    float r;
    asm("v_min_f32 %0, %1, %2" : "=v"(r) : "v"(a), "v"(b));
    return r;
}

template <bool GE>
__global__ __launch_bounds__(64) void k_iou_mask(const float4* __restrict__ boxes, const int32_t* __restrict__ img,
                                                 const int32_t* __restrict__ order, const MaskTask* __restrict__ tasks,
                                                 const int64_t* __restrict__ seg_beg, const int32_t* __restrict__ seg_n,
                                                 const int64_t* __restrict__ seg_mask_off,
                                                 const float* __restrict__ seg_offbase, IouThr th,
                                                 uint64_t* __restrict__ mask, const int32_t* __restrict__ n_tasks) {
  const int T = *n_tasks;  // written by k_nms_plan; the grid is a bound, waves stride over the tasks
  __shared__ float4 cb_box[64];
  __shared__ float cb_area[64];
  for (int ti = blockIdx.x; ti < T; ti += gridDim.x) {
    MaskTask t = tasks[ti];
    const int lane = threadIdx.x;
    const int64_t beg = seg_beg[t.seg];
    const int m = seg_n[t.seg];
    const int nb = (m + 63) >> 6;
    const float ob = seg_offbase[t.seg];
    const int row = t.rb * 64 + lane;
    float4 bi = make_float4(0.f, 0.f, 0.f, 0.f);
    float ai = 0.f;
    if (row < m) {
        bi = load_box(boxes, img, order[beg + row], ob);
        ai = (bi.z - bi.x) * (bi.w - bi.y);
    }
    // layout: word (rb, cb, r) at ((rb * nb + cb) * 64 + r): coalesced writes and scan loads
    uint64_t* out = mask + seg_mask_off[t.seg] + (int64_t)t.rb * nb * 64 + lane;
    // software-pipelined: the next column block's box is loaded while this one is compared
    float4 bnext = make_float4(0.f, 0.f, 0.f, 0.f);
    if (t.cb0 * 64 + lane < m) bnext = load_box(boxes, img, order[beg + t.cb0 * 64 + lane], ob);
    for (int cb = t.cb0; cb < t.cb1; cb++) {
        const float4 bj = bnext;
        if (cb + 1 < t.cb1 && (cb + 1) * 64 + lane < m) bnext = load_box(boxes, img, order[beg + (cb + 1) * 64 + lane], ob);
        __syncthreads();
        cb_box[lane] = bj;
        cb_area[lane] = (bj.z - bj.x) * (bj.w - bj.y);
        __syncthreads();
        const int ncol = min(64, m - cb * 64);
        uint32_t bl = 0, bh = 0, sl = 0, sh = 0;
#pragma unroll
        for (int j = 0; j < 64; j++) {
            const float4 b = cb_box[j];
            // fast path: max / min as v_max / v_min (a NaN coordinate makes uni NaN, and that pair
            // goes to the exact path, which follows the reference's std::max / std::min selects)
            const float xx1 = vmax(bi.x, b.x), yy1 = vmax(bi.y, b.y);
            const float xx2 = vmin(bi.z, b.z), yy2 = vmin(bi.w, b.w);
            const float w = vmax(0.f, xx2 - xx1), h = vmax(0.f, yy2 - yy1);
            const float inter = w * h;
            const float uni = (ai + cb_area[j]) - inter;
            const double l = (double)inter, r = th.mid * (double)uni;
            const uint32_t sup = (GE ? l >= r : l > r) ? 1u : 0u;
            const uint32_t slw = uni > 0.f && uni < INFINITY ? 0u : 1u;
            if (j < 32) bl |= sup << j, sl |= slw << j;
            else bh |= sup << (j - 32), sh |= slw << (j - 32);
        }
        uint64_t bits = ((uint64_t)bh << 32) | bl, slow = ((uint64_t)sh << 32) | sl;
        uint64_t valid = ncol == 64 ? ~0ull : ((1ull << ncol) - 1ull);
        if (cb == t.rb) valid &= lane == 63 ? 0ull : (~0ull << (lane + 1));
        if (row >= m) valid = 0;
        bits &= valid & ~slow;
        slow &= valid;
        while (slow) {  // degenerate unions (rare): the reference's IEEE division
            const int j = __builtin_ctzll(slow);
            slow &= slow - 1;
            const float4 b = cb_box[j];
            // std::max / std::min as the reference writes them ((a < b) ? b : a)
            const float xx1 = bi.x < b.x ? b.x : bi.x, yy1 = bi.y < b.y ? b.y : bi.y;
            const float xx2 = b.z < bi.z ? b.z : bi.z, yy2 = b.w < bi.w ? b.w : bi.w;
            const float dw = xx2 - xx1, dh = yy2 - yy1;
            const float w = 0.f < dw ? dw : 0.f, h = 0.f < dh ? dh : 0.f;
            const float inter = w * h;
            const float ovr = __fdiv_rn(inter, (ai + cb_area[j]) - inter);
            if ((double)ovr > th.thr) bits |= 1ull << j;
        }
        out[(int64_t)cb * 64] = bits;
    }
    __syncthreads();  // cb_box is rewritten by the next task
  }
}

// OR over the 64 lanes with DPP row shifts and row broadcasts (VALU, no LDS crossbar):
// inclusive row scans, then rows folded into lane 63, read back as a wave-uniform value
__device__ inline uint32_t wave_or32(uint32_t v) {
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x111, 0xf, 0xf, true);  // row_shr:1
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x112, 0xf, 0xf, true);  // row_shr:2
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x114, 0xf, 0xf, true);  // row_shr:4
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x118, 0xf, 0xf, true);  // row_shr:8
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x142, 0xa, 0xf, false); // row_bcast:15
    v |= (uint32_t)__builtin_amdgcn_update_dpp(0, (int)v, 0x143, 0xc, 0xf, false); // row_bcast:31
    return (uint32_t)__builtin_amdgcn_readlane((int)v, 63);
}
__device__ inline uint64_t wave_or(uint64_t v) {
    return ((uint64_t)wave_or32((uint32_t)(v >> 32)) << 32) | wave_or32((uint32_t)v);
}

// One workgroup per segment: greedy resolution, 64 rows (one row block) per step, ONE barrier
// per step.  Wave 0 owns the serial chain: it resolves the diagonal 64x64 block of step cb by
// fixed-point iteration (K = alive & ~OR_{q in K} diag_q from K = alive: each round is one wave
// OR; row r's status depends only on rows < r and the greedy keep set is the unique fixed
// point, so the rounds stop at the chain depth -- 2-4 on MTCNN's candidates -- instead of
// visiting every kept row in turn), then ORs its kept rows' words of column block cb + 1 itself
// (the only word the next diagonal needs from this step).  After the barrier the helper waves
// OR the same kept rows' words of column blocks >= cb + 2 into the LDS bitset while wave 0 is
// already on step cb + 1: a column block w is read by wave 0 at step w, and its last helper
// update (step w - 2) finished before the barrier of step w - 1.  Every wave keeps the mask
// words of the next two steps in flight (coalesced 64 rows x 8 B per column block).
constexpr int SCAN_WAVES = 16, SCAN_G = 4;  // helper waves take SCAN_G column blocks each per round
__global__ __launch_bounds__(64 * SCAN_WAVES) void k_nms_scan(const uint64_t* __restrict__ mask,
                                                              const int64_t* __restrict__ seg_beg,
                                                              const int32_t* __restrict__ seg_n,
                                                              const int64_t* __restrict__ seg_mask_off,
                                                              const uint64_t* __restrict__ ck,
                                                              uint64_t* __restrict__ klist, int32_t* __restrict__ kcnt,
                                                              int cap_nb, int32_t* __restrict__ ovf_flag) {
    extern __shared__ uint64_t removed[];
    __shared__ uint64_t s_kept[2];
    constexpr int G = SCAN_G, HW = SCAN_WAVES - 1;
    const int s = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int m = seg_n[s];
    if (m == 0) {
        if (threadIdx.x == 0) kcnt[s] = 0;
        return;
    }
    const int nb = (m + 63) >> 6;
    if (nb > cap_nb) {  // the LDS bitset holds cap_nb words (uniform exit, flag for the host)
        if (threadIdx.x == 0) *ovf_flag = 1, kcnt[s] = 0;
        return;
    }
    const uint64_t* msk = mask + seg_mask_off[s];
    const int64_t beg = seg_beg[s];
    for (int w = threadIdx.x; w < nb; w += 64 * SCAN_WAVES) removed[w] = 0;
    // word (row block rb, column block c, row lane); column blocks past nb - 1 read block nb - 1
    // (never used: the loads stay unconditional and in bounds)
    auto word = [&](int rb, int c) { return msk[((int64_t)rb * nb + min(c, nb - 1)) * 64 + lane]; };
    // wave 0: diagonal and next-column words; helpers: their first-round column words
    uint64_t d1 = 0, x1 = 0, d2 = 0, x2 = 0, v1[G], v2[G];
    auto load = [&](int cb, uint64_t& d, uint64_t& x, uint64_t (&v)[G]) {
        if (wave == 0) {
            d = cb * 64 + lane < m ? word(cb, cb) : 0ull;
            x = word(cb, cb + 1);
        } else {
#pragma unroll
            for (int g = 0; g < G; g++) v[g] = word(cb, cb + 2 + (wave - 1) * G + g);
        }
    };
    load(0, d1, x1, v1);
    if (nb > 1) load(1, d2, x2, v2);
    uint64_t own = 0;  // wave 0: OR of step cb - 1's kept rows over column block cb
    int kpos = 0;      // wave 0: kept rows so far (the segment's kept list is written in order)
    __syncthreads();
    for (int cb = 0; cb < nb; cb++) {
        const uint64_t dg = d1, nx = x1;
        uint64_t v[G];
#pragma unroll
        for (int g = 0; g < G; g++) v[g] = v1[g];
        d1 = d2, x1 = x2;
#pragma unroll
        for (int g = 0; g < G; g++) v1[g] = v2[g];
        if (cb + 2 < nb) load(cb + 2, d2, x2, v2);
        if (wave == 0) {
            const int nrow = min(64, m - cb * 64);
            const uint64_t valid = nrow == 64 ? ~0ull : ((1ull << nrow) - 1ull);
            const uint64_t alive = valid & ~(removed[cb] | own);
            uint64_t kept = alive;
            for (;;) {
                const uint64_t sup = wave_or(((kept >> lane) & 1ull) ? dg : 0ull);
                const uint64_t k2 = alive & ~sup;
                if (k2 == kept) break;
                kept = k2;
            }
            // kept list entry: (descending-score key, element index) -- the order key of the
            // call's output, so k_nms_out can merge a vanilla call's image lists by binary search
            if ((kept >> lane) & 1ull) {
                const int64_t p = beg + cb * 64 + lane;
                klist[beg + kpos + __builtin_popcountll(kept & ((1ull << lane) - 1ull))] = ck[p];
            }
            kpos += __builtin_popcountll(kept);
            if (lane == 0) s_kept[cb & 1] = kept;
            own = wave_or(((kept >> lane) & 1ull) ? nx : 0ull);
        }
        __syncthreads();
        if (wave > 0) {
            const uint64_t kept = s_kept[cb & 1];
            if (kept != 0) {
                const uint64_t mine = ((kept >> lane) & 1ull) ? ~0ull : 0ull;
                for (int w0 = cb + 2 + (wave - 1) * G; w0 < nb; w0 += HW * G) {
                    if (w0 != cb + 2 + (wave - 1) * G) {  // rounds past the first: loaded here
#pragma unroll
                        for (int g = 0; g < G; g++) v[g] = word(cb, w0 + g);
                    }
#pragma unroll
                    for (int g = 0; g < G; g++) {
                        const uint64_t r = wave_or(v[g] & mine);
                        if (lane == 0 && w0 + g < nb) removed[w0 + g] |= r;
                    }
                }
            }
        }
    }
    if (threadIdx.x == 0) kcnt[s] = kpos;
}

// lower bound of key in the sorted list l[0, n)
__device__ inline int lower_bound_u64(const uint64_t* __restrict__ l, int n, uint64_t key) {
    int lo = 0, hi = n;
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (l[mid] < key) lo = mid + 1; else hi = mid;
    }
    return lo;
}

// Output order of every call in one launch: the kept lists (k_nms_scan) already hold each
// segment's kept elements in (score desc, index asc) order.  A coordinate-trick call is one
// segment: its list is its output.  A vanilla call's output is the merge of its image segments'
// lists: an element's rank is its own list index plus, in every other image's list, the count of
// smaller (desc-score key, index) entries (binary search) -- torchvision's final stable-by-index
// score sort.  An equal-score entry with a smaller index in any list of the call flags the call
// for the host's unstable-order fix (torch sorts the vanilla result unstably).  Block 0 also
// writes the per-call kept counts.  koff: exclusive prefix of the kept counts over the segments
// (call-major), recomputed in LDS by every block while S <= NMS_OUT_MAXS; above that (a vanilla
// call over more distinct class ids) k_seg_prefix computes it once into global memory (GK).
constexpr int NMS_OUT_MAXS = 15000;  // (S + 1) x 4 B of dynamic LDS (+ static) within the 64 KB default
constexpr int OUT_G = 16;             // lanes per element: each searches every 16th image list
__global__ __launch_bounds__(256) void k_seg_prefix(const int32_t* __restrict__ kcnt, int S, int32_t* __restrict__ koff) {
    __shared__ int32_t part[256];
    block_prefix<256>(kcnt, S, koff, part);
}
template <bool GK>
__global__ __launch_bounds__(256) void k_nms_out(const uint64_t* __restrict__ klist, const int32_t* __restrict__ kcnt,
                                                 const int64_t* __restrict__ sstart, const uint32_t* __restrict__ seg_hi,
                                                 const int32_t* __restrict__ seg_base, int sbits, int n_img,
                                                 const uint8_t* __restrict__ van, int S, int C, int64_t N,
                                                 int32_t* __restrict__ keep, int32_t* __restrict__ res,
                                                 int32_t* __restrict__ coff, int32_t* __restrict__ dtie,
                                                 const int32_t* __restrict__ koff_g) {
    extern __shared__ int32_t koff_s[];  // [S + 1] (!GK)
    __shared__ int32_t part[256];
    const int tid = threadIdx.x, g = tid & (OUT_G - 1);
    const int32_t* koff = GK ? koff_g : koff_s;
    if (!GK) block_prefix<256>(kcnt, S, koff_s, part);
    if (blockIdx.x == 0)
        for (int c = tid; c <= C; c += 256) {
            if (c < C) res[c] = koff[seg_base[c + 1]] - koff[seg_base[c]];
            coff[c] = koff[seg_base[c]];  // the call's first output position (device copy)
        }
    const int64_t p = ((int64_t)blockIdx.x * 256 + tid) / OUT_G;  // this lane group's element
    if (p >= N) return;  // (uniform over the group)
    int lo = 0, hi = S - 1;  // last segment starting at or before p
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (sstart[mid] <= p) lo = mid; else hi = mid - 1;
    }
    const int sg = lo;
    const int i = (int)(p - sstart[sg]);
    if (i >= kcnt[sg]) return;
    const uint64_t key = klist[p];
    const uint32_t c = seg_hi[sg] >> sbits;
    if (!van[c]) {
        if (g == 0) keep[koff[sg] + i] = (int32_t)(uint32_t)key;
        return;
    }
    const int s0 = seg_base[c];
    int rank = 0;
    bool tie = false;
    for (int t = s0 + g; t < s0 + n_img; t += OUT_G) {
        const int n = kcnt[t];
        if (t == sg || n == 0) continue;
        const uint64_t* l = klist + sstart[t];
        int a = 0, b = n;  // lower bound of key
        while (a < b) {
            const int mid = (a + b) >> 1;
            if (l[mid] < key) a = mid + 1; else b = mid;
        }
        rank += a;
        tie |= a > 0 && (l[a - 1] >> 32) == (key >> 32);
    }
#pragma unroll
    for (int o = 1; o < OUT_G; o <<= 1) {
        rank += __shfl_xor(rank, o, OUT_G);
        tie |= __shfl_xor((int)tie, o, OUT_G) != 0;
    }
    if (g == 0) {
        tie |= i > 0 && (klist[p - 1] >> 32) == (key >> 32);
        keep[koff[s0] + i + rank] = (int32_t)(uint32_t)key;
        if (tie) res[C + 1 + c] = 1, dtie[c] = 1;
    }
}

// The outputs of the calls with equal kept scores (dtie) -> the host mailbox as (element, score)
// pairs: the host reorders them like torch's unstable sort after the call's one sync, and
// k_tie_import writes the order back (no runtime blit copy, no extra sync).
__device__ inline int call_of_output(const int32_t* __restrict__ coff, int C, int q) {
    int lo = 0, hi = C - 1;  // last call starting at or before q
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (coff[mid] <= q) lo = mid; else hi = mid - 1;
    }
    return lo;
}
__global__ void k_tie_export(const int32_t* __restrict__ keep, const float* __restrict__ scores,
                             const int32_t* __restrict__ coff, const int32_t* __restrict__ dtie, int C,
                             int2* __restrict__ mail) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= coff[C]) return;
    if (!dtie[call_of_output(coff, C, q)]) return;
    const int32_t e = keep[q];
    mail[q] = make_int2(e, __float_as_int(scores[e]));
}
__global__ void k_tie_import(const int32_t* __restrict__ mail, const int32_t* __restrict__ coff,
                             const int32_t* __restrict__ dtie, int C, int32_t* __restrict__ keep) {
    const int q = blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= coff[C]) return;
    if (dtie[call_of_output(coff, C, q)]) keep[q] = mail[q];
}

// host staging of several small tables for one H2D copy (16-B aligned members)
struct HostPack {
    std::vector<uint8_t> buf;
    size_t add(const void* p, size_t n) {
        const size_t o = (buf.size() + 15) & ~(size_t)15;
        buf.resize(o + n + 16);
        if (n) std::memcpy(buf.data() + o, p, n);
        buf.resize(o + n);
        return o;
    }
};

// the division-free IoU test's constants for threshold thr (k_iou_mask)
static IouThr iou_thr(double thr) {
    VTF_CHECK(std::isfinite(thr) && std::fabs(thr) < 1e30, VTF_E_ARG, "nms: iou threshold must be finite");
    float f = (float)thr;
    if (!((double)f > thr)) f = std::nextafter(f, INFINITY);  // F: the smallest float above thr
    const float fm = std::nextafter(f, -INFINITY);
    uint32_t bits;
    std::memcpy(&bits, &f, 4);
    return IouThr{thr, ((double)fm + (double)f) * 0.5, (bits & 1u) == 0};
}

static bool nms_debug() {
    static const bool on = [] {
        const char* e = std::getenv("VTF_NMS_DEBUG");
        return e && std::atoi(e) != 0;
    }();
    return on;
}

// Arena slots used here: 40..63 (device), mailboxes 40-43: 40 the call / segment tables, 41 the
// results, 42 the tie export pairs, 43 the host's tie order (k_tie_import reads it after this
// function returns: queued, so mailbox 43 must not be freed meanwhile -- Arena retires grown
// mailboxes instead of freeing them, which keeps the queued read valid)
void nms_multi(Arena& ar, const float* d_boxes, const float* d_scores, const int32_t* d_img,
               const int32_t* d_elem_call, const std::vector<int64_t>& call_n, int n_img, double thr,
               int32_t* d_keep, std::vector<int64_t>& nkeep, hipStream_t st) {
    const int C = (int)call_n.size();
    VTF_CHECK(C < 4096, VTF_E_LIMIT, "nms_multi: too many calls");
    VTF_CHECK(n_img < (1 << 20), VTF_E_LIMIT, "nms_multi: too many images");
    nkeep.assign(C, 0);
    int64_t N = 0;
    std::vector<int64_t> call_beg(C);
    std::vector<uint8_t> vanilla(C);
    std::vector<int32_t> seg_base(C + 1);
    std::vector<int32_t> trick;
    int S = 0;
    for (int c = 0; c < C; c++) {
        call_beg[c] = N;
        N += call_n[c];
        vanilla[c] = call_n[c] * 4 > 4000;
        seg_base[c] = S;
        S += vanilla[c] ? n_img : 1;
        if (!vanilla[c] && call_n[c] > 0) trick.push_back(c);
    }
    seg_base[C] = S;
    if (N == 0) return;
    VTF_CHECK(N < (int64_t)1 << 31, VTF_E_LIMIT, "nms_multi: too many boxes");

    // small host tables (calls, segments) in the handle's pinned mailbox: k_nms_prep copies them
    // to device memory in the same launch that computes the coordinate-trick bases, so there is no
    // runtime blit copy and no memset
    int sbits = 0, cbits = 0;
    while ((1 << sbits) < n_img) sbits++;
    while ((1 << cbits) < C) cbits++;
    std::vector<uint32_t> seg_hi(S);
    for (int c = 0; c < C; c++) {
        for (int s2 = seg_base[c]; s2 < seg_base[c + 1]; s2++) seg_hi[s2] = ((uint32_t)c << sbits) | (uint32_t)(s2 - seg_base[c]);
    }
    HostPack pk;
    const size_t o_cbeg = pk.add(call_beg.data(), C * 8), o_cn = pk.add(call_n.data(), C * 8);
    const size_t o_van = pk.add(vanilla.data(), C), o_sbase = pk.add(seg_base.data(), (C + 1) * 4);
    const size_t o_trick = pk.add(trick.data(), trick.size() * 4), o_seghi = pk.add(seg_hi.data(), S * 4);
    const int tbytes = (int)((pk.buf.size() + 3) & ~(size_t)3);
    Arena::Mail mt = ar.mail(40, tbytes);
    std::memcpy(mt.h, pk.buf.data(), pk.buf.size());
    // results mailbox: kept count per call, the scan's overflow flag (zeroed by k_nms_prep), then
    // a tie flag per call (zeroed by k_nms_prep)
    Arena::Mail mr = ar.mail(41, (size_t)(2 * C + 1) * 4);
    uint8_t* d_t1 = (uint8_t*)ar.get(40, tbytes);
    const int64_t* d_cbeg = (const int64_t*)(d_t1 + o_cbeg);
    const uint8_t* d_van = d_t1 + o_van;
    const uint32_t* d_seghi = (const uint32_t*)(d_t1 + o_seghi);
    const int32_t* d_sbase = (const int32_t*)(d_t1 + o_sbase);
    (void)d_cbeg;
    float* d_cmax = ar.get<float>(52, C);
    int32_t* h_res = (int32_t*)mr.h;
    int32_t* d_res = (int32_t*)mr.d;
    // segmented sort path when every segment fits the LDS sort (a segment holds at most its call's
    // boxes); otherwise the device-wide merge sort
    int64_t segbound = 0;
    for (int c = 0; c < C; c++) segbound = std::max(segbound, call_n[c]);
    // (k_seg_scatter keeps the S + 1 segment offsets in dynamic LDS: 64 KB bound it)
    const bool lds_sort = segbound <= NMS_SORT_BOUND && S < 16000;
    int32_t* d_sctr = ar.get<int32_t>(45, 2 * (size_t)S);
    int32_t* d_tie = ar.get<int32_t>(44, (size_t)2 * C + 1);  // [C] tie flags, [C + 1] call output offsets
    int32_t* d_coff = d_tie + C;
    k_nms_prep<<<1 + (int)trick.size(), 256, 0, st>>>((const uint8_t*)mt.d, d_t1, tbytes, (const float4*)d_boxes, o_cbeg,
                                                      o_cn, o_van, o_trick, C, d_cmax, d_res + C, d_sctr,
                                                      lds_sort ? 2 * S : 0, d_tie);

    // sort 1: (call, segment image, score desc), stable over position order -> ck (desc score key |
    // element index) and ord (element index), segment starts
    uint64_t* k0 = ar.get<uint64_t>(46, N);
    uint64_t* k1 = ar.get<uint64_t>(47, N);
    int32_t* ord = ar.get<int32_t>(49, N);
    int64_t* d_sstart = ar.get<int64_t>(51, (size_t)S + 1);
    uint64_t* ck = k1;
    if (lds_sort) {
        k_seg_count<<<cdiv(N, SEG_T), SEG_T, 0, st>>>(d_img, d_elem_call, d_van, d_sbase, N, S, d_sctr);
        const size_t sc_lds = (size_t)(S + 1 + (S <= SEG_HIST ? 2 * S : 0)) * 4;
        k_seg_scatter<<<cdiv(N, SEG_T), SEG_T, sc_lds, st>>>(d_scores, d_img, d_elem_call, d_van, d_sbase, N, S, d_sctr,
                                                            d_sctr + S, d_sstart, k0);
        k_seg_sort<<<S, 1024, 0, st>>>(d_sstart, k0, k1, ord);
    } else {
        int32_t* v0 = ar.get<int32_t>(48, N);
        k_seg_keys<<<cdiv(N, 256), 256, 0, st>>>(d_scores, d_img, d_elem_call, d_van, N, 1, sbits, k0, v0);
        merge_pairs_u64(ar, 50, k0, k1, v0, ord, N, st);
        // segment bounds by binary search on the sorted keys
        k_seg_bounds<<<cdiv(S + 1, 256), 256, 0, st>>>(k1, N, d_seghi, S, d_sstart);
        ck = k0;
        k_composite<<<cdiv(N, 256), 256, 0, st>>>(k1, ord, N, ck);
    }

    // segment plan + mask tasks on the device (k_nms_plan); the host only sizes buffers and grids
    // from bounds over the calls' counts: a segment of call c has at most call_n[c] boxes, and
    // sum_s nb_s <= call_n / 64 + (segments holding a box)
    int64_t mwords = 0, tbound = 0, nbmax = 0;
    for (int c = 0; c < C; c++) {
        const int64_t n = call_n[c];
        if (n == 0) continue;
        const int64_t nseg = seg_base[c + 1] - seg_base[c];
        const int64_t nbc = (n + 63) / 64, nbsum = n / 64 + std::min(nseg, n);
        nbmax = std::max(nbmax, nbc);
        mwords += nbc * nbsum * 64;          // sum nb_s^2 <= max nb * sum nb
        tbound += nbc * nbsum / 8 + 2 * nbsum + 1;  // ntasks(n) <= n^2 / 8 + 2 n
    }
    int32_t* d_scnt = ar.get<int32_t>(53, S);
    int64_t* d_moff = ar.get<int64_t>(54, S);
    float* d_offb = ar.get<float>(55, S);
    int64_t* d_toff = ar.get<int64_t>(60, (size_t)S + 1);
    MaskTask* d_tasks = ar.get<MaskTask>(62, tbound);
    int32_t* d_ntask = ar.get<int32_t>(63, 1);
    k_nms_plan<<<1, PLAN_T, 0, st>>>(d_sstart, d_seghi, sbits, d_van, d_cmax, S, d_scnt, d_moff, d_offb, d_toff,
                                     d_tasks, d_ntask, tbound);
    uint64_t* d_mask = ar.get<uint64_t>(56, mwords);
    // one wave per task, striding: ~32 waves per CU bound the grid (most tasks cover 8 x 64 x 64 IoUs)
    const IouThr ith = iou_thr(thr);
    const int ig = (int)std::max<int64_t>(1, std::min<int64_t>(tbound, 8192));
    if (ith.ge)
        k_iou_mask<true><<<ig, 64, 0, st>>>((const float4*)d_boxes, d_img, ord, d_tasks, d_sstart, d_scnt, d_moff, d_offb,
                                            ith, d_mask, d_ntask);
    else
        k_iou_mask<false><<<ig, 64, 0, st>>>((const float4*)d_boxes, d_img, ord, d_tasks, d_sstart, d_scnt, d_moff,
                                             d_offb, ith, d_mask, d_ntask);
    uint64_t* d_klist = ar.get<uint64_t>(57, N);
    int32_t* d_kcnt = ar.get<int32_t>(58, S);
    // LDS bitset sized by the largest segment possible (one whole call); a segment beyond the LDS
    // limit raises the mailbox flag instead of overflowing
    const int cap_nb = (int)std::min<int64_t>(nbmax, (160 * 1024 - 64) / 8);  // (+ the static s_kept)
    k_nms_scan<<<S, 64 * SCAN_WAVES, (size_t)cap_nb * 8, st>>>(d_mask, d_sstart, d_scnt, d_moff, ck, d_klist, d_kcnt,
                                                               cap_nb, d_res + C);
    if (nms_debug()) {  // VTF_NMS_DEBUG=1: per-call segment sizes on stderr (synchronises)
        std::vector<int64_t> ss(S + 1);
        VTF_HIP(hipMemcpyAsync(ss.data(), d_sstart, (S + 1) * 8, hipMemcpyDeviceToHost, st));
        VTF_HIP(hipStreamSynchronize(st));
        int64_t mx = 0, pairs = 0, nbs = 0;
        for (int i = 0; i < S; i++) {
            const int64_t m = ss[i + 1] - ss[i], nb = (m + 63) / 64;
            mx = std::max(mx, m);
            pairs += m * (m - 1) / 2;
            nbs += nb;
        }
        fprintf(stderr, "nms_multi: C %d N %lld S %d max seg %lld sum nb %lld pairs %lld\n", C, (long long)N, S,
                (long long)mx, (long long)nbs, (long long)pairs);
    }
    // output order, kept counts and vanilla tie flags in one launch
    if (S <= NMS_OUT_MAXS) {
        k_nms_out<false><<<cdiv(N * OUT_G, 256), 256, (size_t)(S + 1) * 4, st>>>(
            d_klist, d_kcnt, d_sstart, d_seghi, d_sbase, sbits, n_img, d_van, S, C, N, d_keep, d_res, d_coff, d_tie, nullptr);
    } else {
        int32_t* d_koff = ar.get<int32_t>(59, (size_t)S + 1);
        k_seg_prefix<<<1, 256, 0, st>>>(d_kcnt, S, d_koff);
        k_nms_out<true><<<cdiv(N * OUT_G, 256), 256, 0, st>>>(d_klist, d_kcnt, d_sstart, d_seghi, d_sbase, sbits, n_img, d_van,
                                                              S, C, N, d_keep, d_res, d_coff, d_tie, d_koff);
    }
    bool any_van = false;
    for (int c = 0; c < C; c++) any_van |= vanilla[c] != 0;
    int2* h_pairs = nullptr;
    int32_t* d_fix = nullptr;
    if (any_van) {  // flagged calls' outputs to the host, in the same sync
        Arena::Mail mp = ar.mail(42, (size_t)N * 8);
        Arena::Mail mf = ar.mail(43, (size_t)N * 4);
        h_pairs = (int2*)mp.h;
        d_fix = (int32_t*)mf.d;
        k_tie_export<<<cdiv(N, 256), 256, 0, st>>>(d_keep, d_scores, d_coff, d_tie, C, (int2*)mp.d);
        VTF_HIP(hipGetLastError());
    }
    VTF_HIP(hipStreamSynchronize(st));
    VTF_CHECK(h_res[C] == 0, VTF_E_LIMIT, "nms_multi: a segment exceeds 1.3M boxes");
    for (int c = 0; c < C; c++) nkeep[c] = h_res[c];
    // torch's unstable final sort on the vanilla calls with equal kept scores: reordered on the host
    // from the exported pairs, written back by k_tie_import (queued, no sync)
    bool fixed = false;
    int64_t off = 0;
    for (int c = 0; c < C; c++) {
        if (any_van && h_res[C + 1 + c] && nkeep[c] > 1) {
            std::vector<std::pair<int32_t, float>> ps(nkeep[c]);
            for (int64_t t = 0; t < nkeep[c]; t++) ps[t] = {h_pairs[off + t].x, __builtin_bit_cast(float, h_pairs[off + t].y)};
            std::sort(ps.begin(), ps.end(), [](const std::pair<int32_t, float>& a, const std::pair<int32_t, float>& b) {
                return a.first < b.first;
            });
            std::vector<int32_t> hk(nkeep[c]);
            for (int64_t t = 0; t < nkeep[c]; t++) hk[t] = ps[t].first;
            torch_unstable_desc_order(hk, [&](int32_t e) {
                return std::lower_bound(ps.begin(), ps.end(), e, [](const std::pair<int32_t, float>& a, int32_t v) {
                           return a.first < v;
                       })->second;
            });
            int32_t* h_fix = (int32_t*)ar.mptr[43].h;
            std::memcpy(h_fix + off, hk.data(), hk.size() * 4);
            fixed = true;
        }
        off += nkeep[c];
    }
    if (fixed) {
        k_tie_import<<<cdiv(off, 256), 256, 0, st>>>(d_fix, d_coff, d_tie, C, d_keep);
        VTF_HIP(hipGetLastError());
    }
}

}  // namespace vtf

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
// Design (MI355X): a stable merge sort gives every segment's order; an IoU bitmask kernel (one
// wave per 64-row block x column-block chunk, boxes broadcast through LDS) writes u64
// suppression words; one workgroup per segment resolves the greedy chain 64 rows per step
// (fixed-point diagonal in one wave, helper waves OR the kept rows into an LDS bitset, one
// barrier per step).
// Build with -ffp-contract=off: every IoU op is rounded exactly like the CPU kernel.
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <rocprim/device/device_merge_sort.hpp>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

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
                           int C, float* __restrict__ call_max, int32_t* __restrict__ ovf_flag) {
    if (blockIdx.x == 0) {
        if (threadIdx.x == 0) *ovf_flag = 0;
        const uint32_t* src = (const uint32_t*)mail;
        uint32_t* dst = (uint32_t*)tables;
        for (int i = threadIdx.x; i < bytes / 4; i += blockDim.x) dst[i] = src[i];
        const int64_t* cn = (const int64_t*)(mail + o_cn);
        const uint8_t* van = mail + o_van;
        for (int c = threadIdx.x; c < C; c += blockDim.x) {
            if (van[c] || cn[c] == 0) call_max[c] = 0.f;
            ovf_flag[1 + c] = 0;  // tie flags
        }
        return;
    }
    const int c = ((const int32_t*)(mail + o_trick))[blockIdx.x - 1];
    const int64_t beg = ((const int64_t*)(mail + o_cbeg))[c], n = ((const int64_t*)(mail + o_cn))[c];
    float m = -INFINITY;
    for (int64_t i = threadIdx.x; i < n; i += blockDim.x) {
        float4 b = boxes[beg + i];
        m = fmaxf(m, fmaxf(fmaxf(b.x, b.y), fmaxf(b.z, b.w)));
    }
    __shared__ float red[256];
    red[threadIdx.x] = m;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if ((int)threadIdx.x < s) red[threadIdx.x] = fmaxf(red[threadIdx.x], red[threadIdx.x + s]);
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

// One wave per (segment, 64-row block, chunk of column blocks >= rb).
__global__ __launch_bounds__(64) void k_iou_mask(const float4* __restrict__ boxes, const int32_t* __restrict__ img,
                                                 const int32_t* __restrict__ order, const MaskTask* __restrict__ tasks,
                                                 const int64_t* __restrict__ seg_beg, const int32_t* __restrict__ seg_n,
                                                 const int64_t* __restrict__ seg_mask_off,
                                                 const float* __restrict__ seg_offbase, double thr,
                                                 uint64_t* __restrict__ mask, const int32_t* __restrict__ n_tasks) {
  const int T = *n_tasks;  // written by k_nms_plan; the grid is a bound, waves stride over the tasks
  for (int ti = blockIdx.x; ti < T; ti += gridDim.x) {
    MaskTask t = tasks[ti];
    const int lane = threadIdx.x;
    const int64_t beg = seg_beg[t.seg];
    const int m = seg_n[t.seg];
    const int nb = (m + 63) >> 6;
    const float ob = seg_offbase[t.seg];
    const int row = t.rb * 64 + lane;
    __shared__ float4 cb_box[64];
    __shared__ float cb_area[64];
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
        int ncol = min(64, m - cb * 64);
        uint64_t bits = 0;
        if (row < m) {
            int j0 = (cb == t.rb) ? lane + 1 : 0;
            for (int j = j0; j < ncol; j++) {
                float4 b = cb_box[j];
                float xx1 = fmaxf(bi.x, b.x), yy1 = fmaxf(bi.y, b.y);
                float xx2 = fminf(bi.z, b.z), yy2 = fminf(bi.w, b.w);
                float w = fmaxf(0.f, xx2 - xx1), h = fmaxf(0.f, yy2 - yy1);
                float inter = w * h;
                float ovr = __fdiv_rn(inter, (ai + cb_area[j]) - inter);
                if ((double)ovr > thr) bits |= (1ull << j);
            }
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
                                                              uint8_t* __restrict__ keep_sorted, int cap_nb,
                                                              int32_t* __restrict__ ovf_flag) {
    extern __shared__ uint64_t removed[];
    __shared__ uint64_t s_kept[2];
    constexpr int G = SCAN_G, HW = SCAN_WAVES - 1;
    const int s = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int m = seg_n[s];
    if (m == 0) return;
    const int nb = (m + 63) >> 6;
    if (nb > cap_nb) {  // the LDS bitset holds cap_nb words (uniform exit, flag for the host)
        if (threadIdx.x == 0) *ovf_flag = 1;
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
            const int row = cb * 64 + lane;
            if (row < m) keep_sorted[beg + row] = (uint8_t)((kept >> lane) & 1ull);
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
}

__global__ void k_scatter_flags(const int32_t* __restrict__ order, const uint8_t* __restrict__ keep_sorted,
                                int64_t N, uint8_t* __restrict__ keep_elem) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < N) keep_elem[order[k]] = keep_sorted[k];
}

__global__ void k_flag_in_order(const int32_t* __restrict__ order, const uint8_t* __restrict__ keep_elem,
                                int64_t N, int32_t* __restrict__ flag) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k < N) flag[k] = keep_elem[order[k]];
}

__global__ void k_compact(const int32_t* __restrict__ order, const int32_t* __restrict__ flag,
                          const int32_t* __restrict__ incl, int64_t N, int32_t* __restrict__ keep_out) {
    int64_t k = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k >= N || !flag[k]) return;
    keep_out[incl[k] - 1] = order[k];
}

// kept count of call c = incl[end_c - 1] - incl[beg_c - 1], bounds from the sorted keys
__global__ void k_call_kept(const int64_t* __restrict__ call_start, const int32_t* __restrict__ incl, int C,
                            int32_t* __restrict__ out) {
    int c = blockIdx.x * blockDim.x + threadIdx.x;
    if (c >= C) return;
    int64_t b = call_start[c], e = call_start[c + 1];
    int32_t lo = b > 0 ? incl[b - 1] : 0;
    int32_t hi = e > 0 ? incl[e - 1] : 0;
    out[c] = hi - lo;  // (out: the host mailbox)
}

// vanilla calls whose kept set holds two equal scores (adjacent in the stable output order):
// there torch's unstable sort may order them differently, the host reorders that call
__global__ void k_tie_flags(const int32_t* __restrict__ keep, const int32_t* __restrict__ incl, int64_t N,
                            const float* __restrict__ scores, const int32_t* __restrict__ elem_call,
                            const uint8_t* __restrict__ call_van, int32_t* __restrict__ tie) {
    const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x + 1;
    if (N == 0 || p >= incl[N - 1]) return;
    const int32_t a = keep[p - 1], b = keep[p];
    const int32_t c = elem_call[b];
    if (elem_call[a] == c && call_van[c] && scores[a] == scores[b]) tie[c] = 1;  // (tie: the host mailbox)
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

template <class K, class V>
static void radix_pairs(Arena& ar, int slot, const K* kin, K* kout, const V* vin, V* vout, int64_t n, int end_bit,
                        hipStream_t st) {
    size_t tmp = 0;
    VTF_HIP(rocprim::radix_sort_pairs(nullptr, tmp, kin, kout, vin, vout, (size_t)n, 0, end_bit, st));
    void* t = ar.get(slot, tmp);
    VTF_HIP(rocprim::radix_sort_pairs(t, tmp, kin, kout, vin, vout, (size_t)n, 0, end_bit, st));
}

// stable merge sort (block sort + independent merge passes): no decoupled look-back, so it does
// not stall when another lane's persistent kernel holds the CUs (the radix sort's look-back
// blocks waited up to ~0.2 ms per call under 2 lanes); used for nms_multi's two sorts
void merge_pairs_u64(Arena& ar, int slot, const uint64_t* kin, uint64_t* kout, const int32_t* vin,
                            int32_t* vout, int64_t n, hipStream_t st) {
    size_t tmp = 0;
    VTF_HIP(rocprim::merge_sort(nullptr, tmp, kin, kout, vin, vout, (size_t)n, rocprim::less<uint64_t>(), st));
    void* t = ar.get(slot, tmp);
    VTF_HIP(rocprim::merge_sort(t, tmp, kin, kout, vin, vout, (size_t)n, rocprim::less<uint64_t>(), st));
}

void sort_u64_pairs(Arena& ar, int slot, const uint64_t* kin, uint64_t* kout, const int32_t* vin, int32_t* vout,
                    int64_t n, int end_bit, hipStream_t st) {
    radix_pairs(ar, slot, kin, kout, vin, vout, n, end_bit, st);
}

void inclusive_scan_i32(Arena& ar, int slot, const int32_t* in, int32_t* out, int64_t n, hipStream_t st) {
    size_t tmp = 0;
    VTF_HIP(rocprim::inclusive_scan(nullptr, tmp, in, out, (size_t)n, rocprim::plus<int32_t>(), st));
    void* t = ar.get(slot, tmp);
    VTF_HIP(rocprim::inclusive_scan(t, tmp, in, out, (size_t)n, rocprim::plus<int32_t>(), st));
}

static bool nms_debug() {
    static const bool on = [] {
        const char* e = std::getenv("VTF_NMS_DEBUG");
        return e && std::atoi(e) != 0;
    }();
    return on;
}

// Arena slots used here: 40..63 (device), mailboxes 40, 41
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
    std::vector<uint32_t> seg_hi(S), call_hi(C);
    for (int c = 0; c < C; c++) {
        call_hi[c] = (uint32_t)c << sbits;
        for (int s2 = seg_base[c]; s2 < seg_base[c + 1]; s2++) seg_hi[s2] = ((uint32_t)c << sbits) | (uint32_t)(s2 - seg_base[c]);
    }
    HostPack pk;
    const size_t o_cbeg = pk.add(call_beg.data(), C * 8), o_cn = pk.add(call_n.data(), C * 8);
    const size_t o_van = pk.add(vanilla.data(), C), o_sbase = pk.add(seg_base.data(), (C + 1) * 4);
    const size_t o_trick = pk.add(trick.data(), trick.size() * 4), o_seghi = pk.add(seg_hi.data(), S * 4);
    const size_t o_callhi = pk.add(call_hi.data(), C * 4);
    (void)o_sbase;
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
    const uint32_t* d_callhi = (const uint32_t*)(d_t1 + o_callhi);
    (void)d_cbeg;
    float* d_cmax = ar.get<float>(52, C);
    int32_t* h_res = (int32_t*)mr.h;
    int32_t* d_res = (int32_t*)mr.d;
    k_nms_prep<<<1 + (int)trick.size(), 256, 0, st>>>((const uint8_t*)mt.d, d_t1, tbytes, (const float4*)d_boxes, o_cbeg,
                                                      o_cn, o_van, o_trick, C, d_cmax, d_res + C);

    // sort 1: (call, segment image, score desc), stable over position order
    uint64_t* k0 = ar.get<uint64_t>(46, N);
    uint64_t* k1 = ar.get<uint64_t>(47, N);
    int32_t* v0 = ar.get<int32_t>(48, N);
    int32_t* ord = ar.get<int32_t>(49, N);
    k_seg_keys<<<cdiv(N, 256), 256, 0, st>>>(d_scores, d_img, d_elem_call, d_van, N, 1, sbits, k0, v0);
    merge_pairs_u64(ar, 50, k0, k1, v0, ord, N, st);
    // segment bounds by binary search on the sorted keys
    int64_t* d_sstart = ar.get<int64_t>(51, (size_t)S + 1);
    k_seg_bounds<<<cdiv(S + 1, 256), 256, 0, st>>>(k1, N, d_seghi, S, d_sstart);

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
    k_iou_mask<<<(int)std::max<int64_t>(1, std::min<int64_t>(tbound, 8192)), 64, 0, st>>>(
        (const float4*)d_boxes, d_img, ord, d_tasks, d_sstart, d_scnt, d_moff, d_offb, thr, d_mask, d_ntask);
    uint8_t* keep_sorted = ar.get<uint8_t>(57, N);
    // LDS bitset sized by the largest segment possible (one whole call); a segment beyond the LDS
    // limit raises the mailbox flag instead of overflowing
    const int cap_nb = (int)std::min<int64_t>(nbmax, 160 * 1024 / 8);
    k_nms_scan<<<S, 64 * SCAN_WAVES, (size_t)cap_nb * 8, st>>>(d_mask, d_sstart, d_scnt, d_moff, keep_sorted, cap_nb,
                                                               d_res + C);
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
    uint8_t* keep_elem = ar.get<uint8_t>(58, N);
    k_scatter_flags<<<cdiv(N, 256), 256, 0, st>>>(ord, keep_sorted, N, keep_elem);

    // sort 2: (call, score desc), stable over position order -> output order
    k_seg_keys<<<cdiv(N, 256), 256, 0, st>>>(d_scores, d_img, d_elem_call, d_van, N, 0, sbits, k0, v0);
    merge_pairs_u64(ar, 50, k0, k1, v0, ord, N, st);
    int32_t* flag = (int32_t*)k0;  // reuse
    int32_t* incl = ((int32_t*)k0) + N;
    k_flag_in_order<<<cdiv(N, 256), 256, 0, st>>>(ord, keep_elem, N, flag);
    inclusive_scan_i32(ar, 59, flag, incl, N, st);
    k_compact<<<cdiv(N, 256), 256, 0, st>>>(ord, flag, incl, N, d_keep);
    k_seg_bounds<<<cdiv(C + 1, 256), 256, 0, st>>>(k1, N, d_callhi, C, d_sstart);
    k_call_kept<<<cdiv(C, 256), 256, 0, st>>>(d_sstart, incl, C, d_res);
    bool any_van = false;
    for (int c = 0; c < C; c++) any_van |= vanilla[c] != 0;
    if (any_van && N > 1)
        k_tie_flags<<<cdiv(N - 1, 256), 256, 0, st>>>(d_keep, incl, N, d_scores, d_elem_call, d_van, d_res + C + 1);
    VTF_HIP(hipStreamSynchronize(st));
    VTF_CHECK(h_res[C] == 0, VTF_E_LIMIT, "nms_multi: a segment exceeds 1.3M boxes");
    for (int c = 0; c < C; c++) nkeep[c] = h_res[c];
    // torch's unstable final sort on the (rare) vanilla calls with equal kept scores
    int64_t off = 0;
    for (int c = 0; c < C; c++) {
        if (any_van && h_res[C + 1 + c] && nkeep[c] > 1) {
            std::vector<int32_t> hk(nkeep[c]);
            std::vector<float> hs(call_n[c]);
            VTF_HIP(hipMemcpyAsync(hk.data(), d_keep + off, nkeep[c] * 4, hipMemcpyDeviceToHost, st));
            VTF_HIP(hipMemcpyAsync(hs.data(), d_scores + call_beg[c], call_n[c] * 4, hipMemcpyDeviceToHost, st));
            VTF_HIP(hipStreamSynchronize(st));
            const int64_t b = call_beg[c];
            torch_unstable_desc_order(hk, [&](int32_t e) { return hs[e - b]; });
            VTF_HIP(hipMemcpyAsync(d_keep + off, hk.data(), nkeep[c] * 4, hipMemcpyHostToDevice, st));
            VTF_HIP(hipStreamSynchronize(st));
        }
        off += nkeep[c];
    }
}

}  // namespace vtf

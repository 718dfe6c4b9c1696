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
// Design (MI355X): a radix sort gives the stable order; an IoU bitmask kernel (one wave per
// 64-row block, 64x64 tiles, box broadcast through LDS) writes u64 suppression words; a
// single-wave scan per segment resolves the greedy dependence 64 rows at a time in
// registers (readlane) and ORs kept rows into an LDS "removed" bitset -- no barriers.
// Build with -ffp-contract=off: every IoU op is rounded exactly like the CPU kernel.
#include <cstring>
#include <rocprim/device/device_merge_sort.hpp>
#include <rocprim/device/device_radix_sort.hpp>
#include <rocprim/device/device_scan.hpp>

#include <algorithm>

#include "common.hpp"
#include "nms.hpp"

namespace vtf {

__global__ void k_call_max(const float4* __restrict__ boxes, const int64_t* __restrict__ call_beg,
                           const int64_t* __restrict__ call_n, const int32_t* __restrict__ trick_calls,
                           float* __restrict__ call_max) {
    int c = trick_calls[blockIdx.x];
    int64_t beg = call_beg[c], n = call_n[c];
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
                                                 uint64_t* __restrict__ mask) {
    MaskTask t = tasks[blockIdx.x];
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

// One workgroup (8 waves) per segment: greedy resolution, 64 rows per step.  Wave 0 resolves
// the diagonal 64x64 block in registers (readlane); then the kept rows' words of every later
// column block are loaded coalesced (64 rows x 8 B) and OR-reduced across each wave into the LDS
// bitset -- the 8 waves take interleaved groups of column blocks, so 8x the loads are in flight
// (the scan is a serial chain of these steps).
constexpr int SCAN_WAVES = 8;
__global__ __launch_bounds__(64 * SCAN_WAVES) void k_nms_scan(const uint64_t* __restrict__ mask,
                                                              const int64_t* __restrict__ seg_beg,
                                                              const int32_t* __restrict__ seg_n,
                                                              const int64_t* __restrict__ seg_mask_off,
                                                              uint8_t* __restrict__ keep_sorted) {
    extern __shared__ uint64_t removed[];
    __shared__ uint64_t s_kept;
    const int s = blockIdx.x;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int m = seg_n[s];
    if (m == 0) return;
    const int nb = (m + 63) >> 6;
    const uint64_t* msk = mask + seg_mask_off[s];
    const int64_t beg = seg_beg[s];
    for (int w = threadIdx.x; w < nb; w += 64 * SCAN_WAVES) removed[w] = 0;
    // the words a row block needs (its diagonal word and the first round of later column
    // words) are loaded one block ahead, unconditionally: the global-load round trip overlaps the
    // previous block's scan instead of following it (the kept mask is applied after the load)
    constexpr int G = 8;
    auto load_block = [&](int cb, uint64_t& dg, uint64_t (&v)[G]) {
        const uint64_t* blk = msk + (int64_t)cb * nb * 64 + lane;
        dg = (wave == 0 && cb * 64 + lane < m) ? blk[(int64_t)cb * 64] : 0ull;
#pragma unroll
        for (int g = 0; g < G; g++) v[g] = blk[(int64_t)min(cb + 1 + wave * G + g, nb - 1) * 64];
    };
    uint64_t dg_n, v_n[G];
    load_block(0, dg_n, v_n);
    __syncthreads();
    for (int cb = 0; cb < nb; cb++) {
        const uint64_t* blk = msk + (int64_t)cb * nb * 64 + lane;
        const uint64_t diag = dg_n;
        uint64_t v[G];
#pragma unroll
        for (int g = 0; g < G; g++) v[g] = v_n[g];
        if (cb + 1 < nb) load_block(cb + 1, dg_n, v_n);
        if (wave == 0) {
            const int row = cb * 64 + lane;
            const int nrow = min(64, m - cb * 64);
            const uint64_t valid = nrow == 64 ? ~0ull : ((1ull << nrow) - 1ull);
            uint64_t rem = removed[cb];
            uint64_t kept = 0;
            // visit only the rows still alive, in order: each kept row t ORs its diagonal word
            // (lane t, read with a uniform lane index) into the removed set
            uint64_t alive = valid & ~rem;
            while (alive) {
                const int t = __builtin_ctzll(alive);
                const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)diag, t);
                const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(diag >> 32), t);
                kept |= 1ull << t;
                rem |= ((uint64_t)hi << 32) | lo;
                alive = valid & ~rem & (t == 63 ? 0ull : (~0ull << (t + 1)));
            }
            if (row < m) keep_sorted[beg + row] = (uint8_t)((kept >> lane) & 1ull);
            if (lane == 0) s_kept = kept;
        }
        __syncthreads();
        const uint64_t kept = s_kept;
        if (kept != 0) {
            const uint64_t mine = ((kept >> lane) & 1ull) ? ~0ull : 0ull;
            for (int w0 = cb + 1 + wave * G; w0 < nb; w0 += SCAN_WAVES * G) {
                if (w0 != cb + 1 + wave * G) {  // rounds past the first: loaded here
#pragma unroll
                    for (int g = 0; g < G; g++) v[g] = blk[(int64_t)min(w0 + g, nb - 1) * 64];
                }
#pragma unroll
                for (int g = 0; g < G; g++) {
                    const uint64_t r = wave_or(v[g] & mine);
                    if (lane == 0 && w0 + g < nb) removed[w0 + g] |= r;
                }
            }
        }
        __syncthreads();
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
    out[c] = hi - lo;
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

// Arena slots used here: 40..59
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

    // small host->device tables, packed into one transfer (each hipMemcpyAsync from pageable
    // memory is a staged copy + blit kernel: ~4.5 us apiece on the lane's stream)
    int sbits = 0, cbits = 0;
    while ((1 << sbits) < n_img) sbits++;
    while ((1 << cbits) < C) cbits++;
    const int end_bit = 32 + sbits + cbits;
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
    uint8_t* d_t1 = (uint8_t*)ar.get(40, pk.buf.size());
    VTF_HIP(hipMemcpyAsync(d_t1, pk.buf.data(), pk.buf.size(), hipMemcpyHostToDevice, st));
    const int64_t* d_cbeg = (const int64_t*)(d_t1 + o_cbeg);
    const int64_t* d_cn = (const int64_t*)(d_t1 + o_cn);
    const uint8_t* d_van = d_t1 + o_van;
    const uint32_t* d_seghi = (const uint32_t*)(d_t1 + o_seghi);
    const uint32_t* d_callhi = (const uint32_t*)(d_t1 + o_callhi);
    (void)o_sbase;

    // device -> host results of phase 1 share one buffer: segment starts, then call maxima
    uint8_t* d_r1 = (uint8_t*)ar.get(52, (size_t)(S + 1) * 8 + (size_t)C * 4);
    int64_t* d_sstart = (int64_t*)d_r1;
    float* d_cmax = (float*)(d_r1 + (size_t)(S + 1) * 8);
    // per-segment coordinate-trick offset base (max + 1), 0 for vanilla segments
    VTF_HIP(hipMemsetAsync(d_cmax, 0, C * 4, st));
    if (!trick.empty())
        k_call_max<<<(int)trick.size(), 256, 0, st>>>((const float4*)d_boxes, d_cbeg, d_cn,
                                                       (const int32_t*)(d_t1 + o_trick), d_cmax);

    // sort 1: (call, segment image, score desc), stable over position order
    uint64_t* k0 = ar.get<uint64_t>(46, N);
    uint64_t* k1 = ar.get<uint64_t>(47, N);
    int32_t* v0 = ar.get<int32_t>(48, N);
    int32_t* ord = ar.get<int32_t>(49, N);
    k_seg_keys<<<cdiv(N, 256), 256, 0, st>>>(d_scores, d_img, d_elem_call, d_van, N, 1, sbits, k0, v0);
    merge_pairs_u64(ar, 50, k0, k1, v0, ord, N, st);
    (void)end_bit;
    // segment bounds by binary search on the sorted keys
    k_seg_bounds<<<cdiv(S + 1, 256), 256, 0, st>>>(k1, N, d_seghi, S, d_sstart);
    std::vector<uint8_t> r1((size_t)(S + 1) * 8 + (size_t)C * 4);
    VTF_HIP(hipMemcpyAsync(r1.data(), d_r1, r1.size(), hipMemcpyDeviceToHost, st));
    VTF_HIP(hipStreamSynchronize(st));
    const int64_t* sstart = (const int64_t*)r1.data();
    const float* cmax = (const float*)(r1.data() + (size_t)(S + 1) * 8);
    std::vector<int32_t> scnt(S);
    for (int s2 = 0; s2 < S; s2++) scnt[s2] = (int32_t)(sstart[s2 + 1] - sstart[s2]);

    // segment tables, mask offsets, row-block tasks
    std::vector<int64_t> sbeg(S), moff(S);
    std::vector<float> offb(S, 0.f);
    std::vector<MaskTask> tasks;
    int64_t pos = 0, mtot = 0;
    int maxnb = 0;
    for (int c = 0; c < C; c++) {
        for (int s = seg_base[c]; s < seg_base[c + 1]; s++) {
            sbeg[s] = pos;
            moff[s] = mtot;
            int m = scnt[s];
            int nb = (m + 63) / 64;
            maxnb = std::max(maxnb, nb);
            if (!vanilla[c]) offb[s] = cmax[c] + 1.0f;
            for (int rb = 0; rb < nb; rb++)
                for (int c0 = rb; c0 < nb; c0 += MASK_CHUNK) tasks.push_back({s, rb, c0, std::min(nb, c0 + MASK_CHUNK)});
            pos += m;
            mtot += (int64_t)nb * nb * 64;
        }
    }
    VTF_CHECK(maxnb * 8 <= 160 * 1024, VTF_E_LIMIT, "nms_multi: a segment exceeds 1.3M boxes");
    HostPack pk2;
    const size_t o_sbeg = pk2.add(sbeg.data(), S * 8), o_moff = pk2.add(moff.data(), S * 8);
    const size_t o_scnt = pk2.add(scnt.data(), S * 4), o_offb = pk2.add(offb.data(), S * 4);
    const size_t o_tasks = pk2.add(tasks.data(), tasks.size() * sizeof(MaskTask));
    uint8_t* d_t2 = (uint8_t*)ar.get(53, pk2.buf.size());
    VTF_HIP(hipMemcpyAsync(d_t2, pk2.buf.data(), pk2.buf.size(), hipMemcpyHostToDevice, st));
    const int64_t* d_sbeg = (const int64_t*)(d_t2 + o_sbeg);
    const int64_t* d_moff = (const int64_t*)(d_t2 + o_moff);
    const int32_t* d_scnt = (const int32_t*)(d_t2 + o_scnt);
    const float* d_offb = (const float*)(d_t2 + o_offb);
    const MaskTask* d_tasks = (const MaskTask*)(d_t2 + o_tasks);
    uint64_t* d_mask = ar.get<uint64_t>(56, mtot);
    if (!tasks.empty())
        k_iou_mask<<<(int)tasks.size(), 64, 0, st>>>((const float4*)d_boxes, d_img, ord, d_tasks, d_sbeg, d_scnt,
                                                      d_moff, d_offb, thr, d_mask);
    uint8_t* keep_sorted = ar.get<uint8_t>(57, N);
    k_nms_scan<<<S, 64 * SCAN_WAVES, maxnb * 8, st>>>(d_mask, d_sbeg, d_scnt, d_moff, keep_sorted);
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
    int32_t* d_ckept = ar.get<int32_t>(61, C);
    k_call_kept<<<cdiv(C, 256), 256, 0, st>>>(d_sstart, incl, C, d_ckept);
    std::vector<int32_t> ck(C);
    VTF_HIP(hipMemcpyAsync(ck.data(), d_ckept, C * 4, hipMemcpyDeviceToHost, st));
    VTF_HIP(hipStreamSynchronize(st));
    for (int c = 0; c < C; c++) nkeep[c] = ck[c];
}

}  // namespace vtf

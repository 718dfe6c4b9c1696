#pragma once
#include <algorithm>
#include <cmath>
#include <utility>
#include <vector>

#include "common.hpp"

namespace vtf {

// Several independent torchvision batched_nms calls at once.  Elements of call c occupy the
// contiguous range [sum(call_n[<c]), +call_n[c]) of d_boxes/d_scores/d_img, in position order
// (the reference's tensor order).  d_elem_call[e] = c.  Writes the kept element indices of all
// calls to d_keep (call-major, each call in exactly the order torchvision returns: (score desc,
// position asc) -- on the vanilla path (n * 4 > 4000) torch's unstable sort, which differs only
// among equal kept scores: a device check flags such calls and the host reorders just those,
// torch_unstable_desc_order) and their counts to nkeep.  Host-synchronising.
void nms_multi(Arena& ar, const float* d_boxes, const float* d_scores, const int32_t* d_img,
               const int32_t* d_elem_call, const std::vector<int64_t>& call_n, int n_img, double thr,
               int32_t* d_keep, std::vector<int64_t>& nkeep, hipStream_t st);

// torchvision batched_nms above 4000 coordinates (_batched_nms_vanilla, ops/boxes.py) returns
// keep_indices[scores[keep_indices].sort(descending=True)[1]] with keep_indices in index order
// and torch's default (unstable) CPU sort: std::sort of (score, position) pairs with ATen's
// KeyValueCompDesc (aten/src/ATen/native/cpu/SortingKernel.cpp).  Reorders `keep` (element
// indices, any order on entry) into that order; score_of(e) gives element e's score.  Differs
// from the stable (score desc, index asc) order only among equal scores.
template <class F>
inline void torch_unstable_desc_order(std::vector<int32_t>& keep, F score_of) {
    std::sort(keep.begin(), keep.end());
    const int64_t kn = (int64_t)keep.size();
    std::vector<std::pair<float, int64_t>> kv(kn);
    for (int64_t t = 0; t < kn; t++) kv[t] = {score_of(keep[t]), t};
    std::sort(kv.begin(), kv.end(), [](const std::pair<float, int64_t>& a, const std::pair<float, int64_t>& b) {
        return (std::isnan(a.first) && !std::isnan(b.first)) || (a.first > b.first);
    });
    std::vector<int32_t> ord(kn);
    for (int64_t t = 0; t < kn; t++) ord[t] = keep[kv[t].second];
    keep.swap(ord);
}

// prims.hip: (u64 key, i32 value) pairs ascending by (key, value) -- a stable sort by key for
// the callers' position-ordered values -- and an inclusive int32 scan, hand-written (LDS tile
// sort + merge-path passes; tile sums + tile scans): no decoupled look-back (multi-lane friendly)
void merge_pairs_u64(Arena& ar, int slot, const uint64_t* kin, uint64_t* kout, const int32_t* vin, int32_t* vout,
                     int64_t n, hipStream_t st);
void sort_u64_pairs(Arena& ar, int slot, const uint64_t* kin, uint64_t* kout, const int32_t* vin, int32_t* vout,
                    int64_t n, int end_bit, hipStream_t st);
void inclusive_scan_i32(Arena& ar, int slot, const int32_t* in, int32_t* out, int64_t n, hipStream_t st);

}  // namespace vtf

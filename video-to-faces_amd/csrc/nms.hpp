#pragma once
#include <vector>

#include "common.hpp"

namespace vtf {

// Several independent torchvision batched_nms calls at once.  Elements of call c occupy the
// contiguous range [sum(call_n[<c]), +call_n[c]) of d_boxes/d_scores/d_img, in position order
// (the reference's tensor order).  d_elem_call[e] = c.  Writes the kept element indices of all
// calls to d_keep (call-major, each call in (score desc, position asc) order, i.e. exactly the
// order torchvision returns) and their counts to nkeep.  Host-synchronising.
void nms_multi(Arena& ar, const float* d_boxes, const float* d_scores, const int32_t* d_img,
               const int32_t* d_elem_call, const std::vector<int64_t>& call_n, int n_img, double thr,
               int32_t* d_keep, std::vector<int64_t>& nkeep, hipStream_t st);

// stable merge sort of (u64 key, i32 value) pairs, no decoupled look-back (multi-lane friendly)
void merge_pairs_u64(Arena& ar, int slot, const uint64_t* kin, uint64_t* kout, const int32_t* vin, int32_t* vout,
                     int64_t n, hipStream_t st);
void sort_u64_pairs(Arena& ar, int slot, const uint64_t* kin, uint64_t* kout, const int32_t* vin, int32_t* vout,
                    int64_t n, int end_bit, hipStream_t st);
void inclusive_scan_i32(Arena& ar, int slot, const int32_t* in, int32_t* out, int64_t n, hipStream_t st);

}  // namespace vtf

#pragma once
#include <vector>

#include "common.hpp"

namespace vtf {

// Detector rows -> face crop rectangles on device (detection.py:133-145: filter_boxes 174-217,
// adjust_boxes 220-262, the (frame, face) flatten of get_crops 161-162).
// d_rows [n,5] fp32 (x1,y1,x2,y2,score) grouped by frame, d_counts [B] rows per frame (device).
// Writes the kept crops d_crops [m,5] int32 (frame_offset + frame, x1, y1, x2, y2) in row order,
// d_src [m] (row index of each crop, may be null), d_frame_counts [B] and d_total [1].
// One workgroup: a det-batch holds at most a few thousand rows.
constexpr int BOX_MAX_FRAMES = 4096;
void launch_box_post(const float* d_rows, const int32_t* d_counts, int B, int H, int W, const vtf_box_params& p,
                     int frame_offset, int32_t* d_crops, int32_t* d_src, int32_t* d_frame_counts, int32_t* d_total,
                     hipStream_t st, int64_t cap = INT64_MAX);

// launch_box_post on a detector's device rows with host per-frame counts (negative = the frame is
// absent from the detector's output, as R-CNN past its last proposal image: no crops).  Uploads the
// counts, reads back the total (one sync).  Fails with VTF_E_CAPACITY (*out_n = rows) when the
// rows exceed `cap` crops.  h_frame_counts (may be null) receives the kept crops per frame.
int64_t rows_to_crops(Arena& ar, int slot, const float* d_rows, const std::vector<int32_t>& counts, int H, int W,
                      const vtf_box_params& p, int frame_offset, int32_t* d_crops, int32_t* d_src,
                      int32_t* h_frame_counts, int64_t cap, int64_t* out_n, hipStream_t st);

// Host-side validation of crop rectangles handed to an encoder (frame index and slice bounds).
void check_crops_host(const int32_t* crops, int64_t N, int F, int H, int W);

}  // namespace vtf

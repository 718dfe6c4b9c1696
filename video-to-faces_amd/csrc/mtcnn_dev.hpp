// Device helpers shared by the MTCNN kernels (mtcnn_kernels.hip, mtcnn_cand.hip).
#pragma once
#include "common.hpp"

namespace vtf {

// adaptive_avg_pool2d bin of the preprocessed frame (x - 127.5) / 128 = (2u - 255) / 256 from an
// exact integer box sum: fp32 sum, then / kh, then / kw, as the reference CPU kernel divides
__device__ inline float bin_avg(int sum, int kh, int kw) {
    return __fdiv_rn(__fdiv_rn((float)sum * 0.00390625f, (float)kh), (float)kw);
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

}  // namespace vtf

#pragma once
#include "common.hpp"

namespace vtf {
// layout 0: NCHW fp32 [N,3,S,S]; layout 1: NHWC [N,S,S,Cp] fp32 or bf16
void launch_blob(const uint8_t* frames, int H, int W, int64_t fstride, int64_t rstride, const int32_t* d_crops,
                 int64_t N, int S, float mean, float scale, int layout, int Cp, bool bf16, void* out, hipStream_t st);
}

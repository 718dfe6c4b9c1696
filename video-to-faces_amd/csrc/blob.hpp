#pragma once
#include "common.hpp"

namespace vtf {
// OpenCV INTER_LINEAR (uint8) coefficients for destination index d (blob.hip header).
__device__ inline void lin_coef(int d, int src, int dst, int& s0, int& s1, int& c0, int& c1, bool& edge) {
    double scale = 1.0 / ((double)dst / (double)src);
    float f = (float)(((double)d + 0.5) * scale - 0.5);
    int s = (int)floorf(f);
    f -= (float)s;
    edge = false;
    if (s < 0) {
        f = 0.f;
        s = 0;
    }
    if (s >= src - 1) {
        f = 0.f;
        s = src - 1;
        edge = true;
    }
    s0 = s;
    s1 = min(s + 1, src - 1);
    c0 = (int)rintf((1.f - f) * 2048.f);
    c1 = (int)rintf(f * 2048.f);
}

// layout 0: NCHW fp32 [N,3,S,S]; layout 1: NHWC [N,S,S,Cp] fp32 or bf16
void launch_blob(const uint8_t* frames, int F, int H, int W, int64_t fstride, int64_t rstride, const int32_t* d_crops,
                 int64_t N, int S, float mean, float scale, int layout, int Cp, bool bf16, void* out, hipStream_t st);
}

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

// the crop img[y1:y2, x1:x2] of frame f (crops row [f, x1, y1, x2, y2]) with numpy slice
// semantics for in-frame boxes; a frame index outside [0, F) gives an empty crop (a zero image)
__device__ inline const uint8_t* blob_crop(const uint8_t* frames, int F, int H, int W, int64_t fstride, int64_t rstride,
                                           const int32_t* c, int& w, int& h) {
    const int f = c[0];
    int x1 = c[1], y1 = c[2], x2 = c[3], y2 = c[4];
    x1 = max(0, min(x1, W));
    x2 = max(x1, min(x2, W));
    y1 = max(0, min(y1, H));
    y2 = max(y1, min(y2, H));
    w = x2 - x1;
    h = y2 - y1;
    if (f < 0 || f >= F) w = h = 0;
    return frames + (int64_t)(w > 0 && h > 0 ? f : 0) * fstride + (int64_t)y1 * rstride + (int64_t)x1 * 3;
}

// one channel of the INTER_LINEAR pixel from source rows r0 / r1 and the column / row
// coefficients of lin_coef (OpenCV's integer rounding, blob.hip header)
__device__ inline int blob_lin(const uint8_t* r0, const uint8_t* r1, int sx0, int sx1, int a0, int a1, bool ex, int b0,
                               int b1, int ch) {
    const int h0 = ex ? r0[sx0 * 3 + ch] * 2048 : r0[sx0 * 3 + ch] * a0 + r0[sx1 * 3 + ch] * a1;
    const int h1 = ex ? r1[sx0 * 3 + ch] * 2048 : r1[sx0 * 3 + ch] * a0 + r1[sx1 * 3 + ch] * a1;
    int t = (((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16);
    t = (t + 2) >> 2;
    return min(255, max(0, t));
}

// layout 0: NCHW fp32 [N,3,S,S]; layout 1: NHWC [N,S,S,Cp] fp32 or bf16
void launch_blob(const uint8_t* frames, int F, int H, int W, int64_t fstride, int64_t rstride, const int32_t* d_crops,
                 int64_t N, int S, float mean, float scale, int layout, int Cp, bool bf16, void* out, hipStream_t st);
}

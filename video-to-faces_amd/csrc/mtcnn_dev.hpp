// Device helpers shared by the MTCNN kernels (mtcnn_kernels.hip, mtcnn_cand.hip).
#pragma once
#include <type_traits>

#include "common.hpp"

namespace vtf {

// adaptive_avg_pool2d bin of the preprocessed frame (x - 127.5) / 128 = (2u - 255) / 256 from an
// exact integer box sum: fp32 sum, then / kh, then / kw, as the reference CPU kernel divides
__device__ inline float bin_avg(int sum, int kh, int kw) {
    return __fdiv_rn(__fdiv_rn((float)sum * 0.00390625f, (float)kh), (float)kw);
}

__device__ inline float prelu(float x, float a) { return x > 0.f ? x : a * x; }

// The det-batch's summed-area table comes in two layouts at the same element indices
// [B][H + 1][W + 1] (sums over rows < y, cols < x):
//   int3:   v = 2u - 255 sums (R, G, B), 12 B per entry;
//   packed: uint64 prefix sums, mod 2^64, of u_R | u_G << 21 | u_B << 42 (8 B per entry).  The
//           four-corner combination d - b - c + a of a box is then sum_c box_c 2^(21 c) mod 2^64,
//           exact field by field while every channel's box sum of u is below 2^21, i.e. for boxes
//           of at most 8223 pixels (the host checks every bin a det-batch reads: sat_pack_ok).
__device__ inline uint64_t sat_pack_px(const uint8_t* bgr) {
    return (uint64_t)bgr[2] | (uint64_t)bgr[1] << 21 | (uint64_t)bgr[0] << 42;
}

// v = 2u - 255 box sums (R, G, B) from packed corners a (top-left), b (top-right), c, d
__device__ inline int3 sat_box_pk(uint64_t a, uint64_t b, uint64_t c, uint64_t d, int area) {
    const uint64_t t = d - b - c + a;
    const int m = (1 << 21) - 1, z = 255 * area;
    return make_int3(2 * (int)(t & m) - z, 2 * (int)((t >> 21) & m) - z, 2 * (int)((t >> 42) & m) - z);
}

__device__ inline int3 sat_box_i3(int3 a, int3 b, int3 c, int3 d) {
    return make_int3(d.x - b.x - c.x + a.x, d.y - b.y - c.y + a.y, d.z - b.z - c.z + a.z);
}

// box rows [ys, ye) x cols [xs, xe) of the table at element offset `base` (row length W1)
__device__ inline int3 sat_box_any(const void* sat, int pk, int64_t base, int64_t W1, int ys, int ye, int xs, int xe) {
    const int64_t ra = base + ys * W1, rb = base + ye * W1;
    if (pk) {
        const uint64_t* q = (const uint64_t*)sat;
        return sat_box_pk(q[ra + xs], q[ra + xe], q[rb + xs], q[rb + xe], (ye - ys) * (xe - xs));
    }
    const int3* q = (const int3*)sat;
    return sat_box_i3(q[ra + xs], q[ra + xe], q[rb + xs], q[rb + xe]);
}

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

// bins idx[j] (row-major in an S x S grid) of the adaptive-pool crop of the frame box at rows
// y0 .. y0 + hc, cols x0 .. x0 + wc, from the table at element offset `base` (row length W1):
// v-sums and bin sizes.  Every corner load is issued before any is combined (the gathers are
// latency-bound: 4 N loads in flight per thread).
template <int N, int S, bool PK>
__device__ inline void crop_bins(const void* sat, int64_t base, int64_t W1, int y0, int x0, int hc, int wc,
                                 const int (&idx)[N], int3 (&sum)[N], int (&kh)[N], int (&kw)[N]) {
    typedef typename std::conditional<PK, uint64_t, int3>::type T;
    const T* q = (const T*)sat;
    T cn[N][4];
#pragma unroll
    for (int j = 0; j < N; j++) {
        const int r = idx[j] / S, c = idx[j] - r * S;
        const int ys = (r * hc) / S, ye = ((r + 1) * hc + S - 1) / S;
        const int xs = (c * wc) / S, xe = ((c + 1) * wc + S - 1) / S;
        kh[j] = ye - ys;
        kw[j] = xe - xs;
        const int64_t ra = base + (int64_t)(y0 + ys) * W1 + x0, rb = base + (int64_t)(y0 + ye) * W1 + x0;
        cn[j][0] = q[ra + xs];
        cn[j][1] = q[ra + xe];
        cn[j][2] = q[rb + xs];
        cn[j][3] = q[rb + xe];
    }
#pragma unroll
    for (int j = 0; j < N; j++) {
        if constexpr (PK)
            sum[j] = sat_box_pk(cn[j][0], cn[j][1], cn[j][2], cn[j][3], kh[j] * kw[j]);
        else
            sum[j] = sat_box_i3(cn[j][0], cn[j][1], cn[j][2], cn[j][3]);
    }
}

}  // namespace vtf

// Decoded-video frames -> the detectors' BGR frames in HBM (the reference's
// frame source is process_video, src/videotofaces/detection.py:68-111: cv2.VideoCapture /
// decord hand it uint8 BGR [B,H,W,3] frames).
//
// The image has no video codec (no cv2, decord, FFmpeg or rocDecode), so the decode boundary here
// is raw planar YUV -- the YUV4MPEG2 stream any decoder can emit (videotofaces/video.py parses
// the container and uploads each sampled frame's planes as they lie in the file: 1.5 bytes per
// pixel over PCIe for 4:2:0 instead of 3) -- and the colour conversion runs on the GPU:
//
//   k_yuv420_to_bgr_8x2 (4:2:0, W % 8 == 0: one thread per 8 x 2 block, 8-byte accesses) or
//   k_yuv_to_bgr (any layout: one thread per 4 pixels of a row, 4-byte accesses when W % 4 == 0
//   and the strides allow); chroma sampled nearest (each
//   4:2:0 chroma sample covers its 2 x 2 luma block, as cv2.cvtColor(COLOR_YUV2BGR_I420) reads
//   it) and the BT.601 integer transform with 20 fractional bits:
//     limited range: y = max(0, Y - 16) * 1220542,  R = (y + 2^19 + 1673527 V') >> 20,
//                    G = (y + 2^19 - 852492 V' - 409993 U') >> 20,  B = (y + 2^19 + 2116026 U') >> 20
//     full range:    y = Y << 20,  R = (y + 2^19 + 1470104 V') >> 20,
//                    G = (y + 2^19 - 748826 V' - 360853 U') >> 20,  B = (y + 2^19 + 1858077 U') >> 20
//   (U' = U - 128, V' = V - 128, saturated to [0, 255]; the limited-range constants are OpenCV's
//   ITUR_BT_601_* ones).  HBM-bound: 1.5 B read + 3 B written per 4:2:0 pixel.
// cv2 / FFmpeg are absent: which conversion the reference's VideoCapture applies (swscale's) is
// parity-UNPINNED; the kernel is pinned to its own restatement (oracle/yuv.py) bit for bit.
#include "common.hpp"

namespace vtf {

namespace {

struct YuvGeom {
    int H, W, sx, sy, cw, ch;  // chroma subsampling shifts and plane size
    int full;
    int64_t in_stride, out_fstride, out_rstride;
};

// (x >> 20) saturated to [0, 255], materialised as a 32-bit value: the empty asm keeps the
// compiler from fusing shift + saturate + byte packing into v_ashr_pk_u8_i32, whose packed result
// was OR-ed with the neighbouring bytes as if its upper half were zero -- measured wrong bytes 2 / 3
// of the packed words on the GPU (ROCm 7.2 hipcc, gfx950)
__device__ inline uint8_t sat_u8(int x) {
    int v = min(255, max(0, x >> 20));
    asm volatile("" : "+v"(v));
    return (uint8_t)v;
}

template <bool FULL>
__device__ inline void yuv_px(int Y, int U, int V, uint8_t& b, uint8_t& g, uint8_t& r) {
    const int u = U - 128, v = V - 128;
    const int y = (FULL ? Y << 20 : max(0, Y - 16) * 1220542) + (1 << 19);
    const int cr = FULL ? 1470104 : 1673527, cgv = FULL ? -748826 : -852492;
    const int cgu = FULL ? -360853 : -409993, cb = FULL ? 1858077 : 2116026;
    r = sat_u8(y + cr * v);
    g = sat_u8(y + cgv * v + cgu * u);
    b = sat_u8(y + cb * u);
}

__device__ inline uint32_t pack4(const uint8_t* q) {
    return (uint32_t)q[0] | (uint32_t)q[1] << 8 | (uint32_t)q[2] << 16 | (uint32_t)q[3] << 24;
}

// VEC: W % 4 == 0 and every stride a multiple of 4 -> one 4-byte luma load, three 4-byte stores
template <bool VEC, bool FULL>
__global__ __launch_bounds__(256) void k_yuv_to_bgr(const uint8_t* __restrict__ in, int64_t n, YuvGeom g,
                                                    uint8_t* __restrict__ out) {
    const int qw = (g.W + 3) >> 2;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t per = (int64_t)g.H * qw;
    if (i >= n * per) return;
    const int64_t f = i / per;
    const int rem = (int)(i - f * per);
    const int y = rem / qw, x0 = (rem - y * qw) * 4;
    const uint8_t* Yp = in + f * g.in_stride;
    const uint8_t* Up = Yp + (int64_t)g.H * g.W;
    const uint8_t* Vp = Up + (int64_t)g.cw * g.ch;
    const bool mono = g.cw == 0;
    const int crow = (y >> g.sy) * g.cw;
    uint8_t* o = out + f * g.out_fstride + (int64_t)y * g.out_rstride + (int64_t)x0 * 3;
    uint8_t px[12];
    uint32_t yv = 0;
    if (VEC) yv = *(const uint32_t*)(Yp + (int64_t)y * g.W + x0);
#pragma unroll
    for (int k = 0; k < 4; k++) {
        const int x = x0 + k;
        if (!VEC && x >= g.W) break;
        const int Y = VEC ? (int)((yv >> (8 * k)) & 255u) : Yp[(int64_t)y * g.W + x];
        const int U = mono ? 128 : Up[crow + (x >> g.sx)];
        const int V = mono ? 128 : Vp[crow + (x >> g.sx)];
        yuv_px<FULL>(Y, U, V, px[3 * k], px[3 * k + 1], px[3 * k + 2]);
        if (!VEC) o[3 * k] = px[3 * k], o[3 * k + 1] = px[3 * k + 1], o[3 * k + 2] = px[3 * k + 2];
    }
    if (VEC) {
        uint32_t* o4 = (uint32_t*)o;
        o4[0] = pack4(px), o4[1] = pack4(px + 4), o4[2] = pack4(px + 8);
    }
}

// 4:2:0 with W % 8 == 0 and 8-byte aligned planes / strides: one thread per 8 x 2 pixel block --
// two 8-byte luma loads, one 4-byte load per chroma plane (the block's 4 x 1 chroma samples),
// six 8-byte stores
template <bool FULL>
__global__ __launch_bounds__(256) void k_yuv420_to_bgr_8x2(const uint8_t* __restrict__ in, int64_t n, YuvGeom g,
                                                           uint8_t* __restrict__ out) {
    const int gw = g.W >> 3, rp = (g.H + 1) >> 1;
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    const int64_t per = (int64_t)rp * gw;
    if (i >= n * per) return;
    const int64_t f = i / per;
    const int rem = (int)(i - f * per);
    const int r = rem / gw, x0 = (rem - r * gw) * 8;
    const uint8_t* Yp = in + f * g.in_stride;
    const uint8_t* Up = Yp + (int64_t)g.H * g.W;
    const uint8_t* Vp = Up + (int64_t)g.cw * g.ch;
    const uint32_t uv = *(const uint32_t*)(Up + r * g.cw + (x0 >> 1));
    const uint32_t vv = *(const uint32_t*)(Vp + r * g.cw + (x0 >> 1));
#pragma unroll
    for (int h = 0; h < 2; h++) {
        const int y = 2 * r + h;
        if (y >= g.H) break;
        const uint64_t yv = *(const uint64_t*)(Yp + (int64_t)y * g.W + x0);
        uint8_t px[24];
#pragma unroll
        for (int k = 0; k < 8; k++)
            yuv_px<FULL>((int)((yv >> (8 * k)) & 255u), (int)((uv >> (8 * (k >> 1))) & 255u),
                         (int)((vv >> (8 * (k >> 1))) & 255u), px[3 * k], px[3 * k + 1], px[3 * k + 2]);
        uint64_t* o = (uint64_t*)(out + f * g.out_fstride + (int64_t)y * g.out_rstride + (int64_t)x0 * 3);
#pragma unroll
        for (int j = 0; j < 3; j++) o[j] = (uint64_t)pack4(px + 8 * j) | (uint64_t)pack4(px + 8 * j + 4) << 32;
    }
}

}  // namespace

}  // namespace vtf

using namespace vtf;

extern "C" int vtf_yuv_to_bgr(const uint8_t* d_yuv, int64_t n, int H, int W, int chroma, int full_range,
                              int64_t in_frame_stride, uint8_t* d_bgr, int64_t out_frame_stride,
                              int64_t out_row_stride, void* hip_stream) {
    return guarded_on(stream_device((hipStream_t)hip_stream), [&] {
        VTF_CHECK(n >= 0 && H > 0 && W > 0, VTF_E_ARG, "yuv_to_bgr: bad size");
        VTF_CHECK(chroma == 420 || chroma == 422 || chroma == 444 || chroma == 400, VTF_E_ARG,
                  "yuv_to_bgr: chroma must be 420, 422, 444 or 400 (mono)");
        if (n == 0) return;
        VTF_CHECK(d_yuv && d_bgr, VTF_E_ARG, "null argument");
        YuvGeom g{};
        g.H = H, g.W = W;
        g.sx = chroma == 444 ? 0 : 1;
        g.sy = chroma == 420 ? 1 : 0;
        g.cw = chroma == 400 ? 0 : (W + g.sx) >> g.sx;
        g.ch = chroma == 400 ? 0 : (H + g.sy) >> g.sy;
        g.full = full_range != 0;
        const int64_t need = (int64_t)H * W + 2 * (int64_t)g.cw * g.ch;
        VTF_CHECK(in_frame_stride >= need, VTF_E_ARG, "yuv_to_bgr: input frame stride below the plane bytes");
        VTF_CHECK(out_row_stride >= (int64_t)W * 3 && out_frame_stride >= out_row_stride * H, VTF_E_ARG,
                  "yuv_to_bgr: output strides");
        g.in_stride = in_frame_stride, g.out_fstride = out_frame_stride, g.out_rstride = out_row_stride;
        const int64_t items = n * H * (int64_t)((W + 3) / 4);
        VTF_CHECK(items / 256 < (int64_t)1 << 31, VTF_E_LIMIT, "yuv_to_bgr: too many frames in one call");
        hipStream_t st = (hipStream_t)hip_stream;
        const bool v8 = chroma == 420 && W % 8 == 0 && in_frame_stride % 8 == 0 && out_frame_stride % 8 == 0 &&
                        out_row_stride % 8 == 0 && ((uintptr_t)d_yuv & 7) == 0 && ((uintptr_t)d_bgr & 7) == 0;
        if (v8) {
            const int64_t blocks = n * ((H + 1) / 2) * (int64_t)(W / 8);
            const unsigned grid8 = (unsigned)((blocks + 255) / 256);
            if (g.full)
                k_yuv420_to_bgr_8x2<true><<<grid8, 256, 0, st>>>(d_yuv, n, g, d_bgr);
            else
                k_yuv420_to_bgr_8x2<false><<<grid8, 256, 0, st>>>(d_yuv, n, g, d_bgr);
            VTF_HIP(hipGetLastError());
            return;
        }
        const bool vec = W % 4 == 0 && in_frame_stride % 4 == 0 && out_frame_stride % 4 == 0 && out_row_stride % 4 == 0 &&
                         ((uintptr_t)d_yuv & 3) == 0 && ((uintptr_t)d_bgr & 3) == 0;
        const unsigned grid = (unsigned)((items + 255) / 256);
        if (vec && g.full)
            k_yuv_to_bgr<true, true><<<grid, 256, 0, st>>>(d_yuv, n, g, d_bgr);
        else if (vec)
            k_yuv_to_bgr<true, false><<<grid, 256, 0, st>>>(d_yuv, n, g, d_bgr);
        else if (g.full)
            k_yuv_to_bgr<false, true><<<grid, 256, 0, st>>>(d_yuv, n, g, d_bgr);
        else
            k_yuv_to_bgr<false, false><<<grid, 256, 0, st>>>(d_yuv, n, g, d_bgr);
        VTF_HIP(hipGetLastError());
    });
}

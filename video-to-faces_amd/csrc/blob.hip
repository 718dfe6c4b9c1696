// cv2.dnn.blobFromImages on device crops (src/videotofaces/encoders/facenet.py:179,
// encoders/vit.py:141): each face crop (a slice of a frame in HBM, detection.py:161-162) is
// resized to S x S with OpenCV's uint8 INTER_LINEAR, converted to float, mean-subtracted,
// scaled and written RGB (swapRB).  This replaces the reference's JPEG write/read round trip
// between detection and encoding (detection.py:156 -> grouping.py:34).
//
// INTER_LINEAR restated from OpenCV's published resize (resizeGeneric_ with
// HResizeLinear + the SIMD VResizeLinearVec_32s8u rounding):
//   fx = (float)((dx + 0.5) * (src/dst) - 0.5); sx = floor(fx); fx -= sx; clamp sx to
//   [0, w-1] with fx = 0 at the borders; a0 = rint((1-fx)*2048), a1 = rint(fx*2048);
//   h = S[sx]*a0 + S[sx+1]*a1 (or S[w-1]*2048 at the right border); same for rows;
//   out = ((((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16) + 2) >> 2, saturated.
// cv2 is not installed here, so this step is parity-UNPINNED (tests pin the post-blob
// tensor -> embedding boundary instead).
#include "common.hpp"
#include "blob.hpp"

namespace vtf {

template <typename T>
__device__ inline T cvt_out(float v);
template <>
__device__ inline float cvt_out<float>(float v) { return v; }
template <>
__device__ inline __bf16 cvt_out<__bf16>(float v) { return (__bf16)v; }

// layout 0: NCHW [N,3,S,S]; layout 1: NHWC [N,S,S,Cp] (channels >= 3 zero)
template <typename T, int LAYOUT>
__global__ void k_blob(const uint8_t* __restrict__ frames, int F, int H, int W, int64_t fstride, int64_t rstride,
                       const int32_t* __restrict__ crops, int64_t N, int S, float mean, float scale, int Cp,
                       T* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N * S * S) return;
    int dx = (int)(i % S);
    int dy = (int)((i / S) % S);
    int64_t n = i / ((int64_t)S * S);
    int w, h;
    const uint8_t* base = blob_crop(frames, F, H, W, fstride, rstride, crops + n * 5, w, h);
    int v[3];
    if (w <= 0 || h <= 0) {
        v[0] = v[1] = v[2] = 0;
    } else if (w == S && h == S) {
        const uint8_t* p = base + (int64_t)dy * rstride + dx * 3;
        v[0] = p[0];
        v[1] = p[1];
        v[2] = p[2];
    } else {
        int sx0, sx1, a0, a1, sy0, sy1, b0, b1;
        bool ex, ey;
        lin_coef(dx, w, S, sx0, sx1, a0, a1, ex);
        lin_coef(dy, h, S, sy0, sy1, b0, b1, ey);
        (void)ey;
        const uint8_t* r0 = base + (int64_t)sy0 * rstride;
        const uint8_t* r1 = base + (int64_t)sy1 * rstride;
#pragma unroll
        for (int ch = 0; ch < 3; ch++) v[ch] = blob_lin(r0, r1, sx0, sx1, a0, a1, ex, b0, b1, ch);
    }
    // swapRB: output channel 0 = R = BGR byte 2
    if (LAYOUT == 1 && Cp == 8) {
        // the pixel's 8 channels (3 values, 5 zeros) as one vector store (16 B bf16 / 32 B fp32)
        // instead of eight scalar ones
        T px[8];
#pragma unroll
        for (int oc = 0; oc < 8; oc++) px[oc] = cvt_out<T>(oc < 3 ? ((float)v[2 - oc] - mean) * scale : 0.f);
        T* o = out + ((n * S + dy) * S + dx) * 8;
        if constexpr (sizeof(T) == 2) {
            *(uint4*)o = __builtin_bit_cast(uint4, px);
        } else {
            ((uint4*)o)[0] = make_uint4(__float_as_uint(px[0]), __float_as_uint(px[1]), __float_as_uint(px[2]), __float_as_uint(px[3]));
            ((uint4*)o)[1] = make_uint4(0u, 0u, 0u, 0u);
        }
        return;
    }
    for (int oc = 0; oc < 3; oc++) {
        float val = ((float)v[2 - oc] - mean) * scale;
        if (LAYOUT == 0)
            out[((n * 3 + oc) * S + dy) * S + dx] = cvt_out<T>(val);
        else
            out[((n * S + dy) * S + dx) * Cp + oc] = cvt_out<T>(val);
    }
    if (LAYOUT == 1)
        for (int oc = 3; oc < Cp; oc++) out[((n * S + dy) * S + dx) * Cp + oc] = cvt_out<T>(0.f);
}

void launch_blob(const uint8_t* frames, int F, int H, int W, int64_t fstride, int64_t rstride, const int32_t* d_crops,
                 int64_t N, int S, float mean, float scale, int layout, int Cp, bool bf16, void* out, hipStream_t st) {
    int64_t tot = N * S * S;
    if (tot <= 0) return;
    if (layout == 0)
        k_blob<float, 0><<<cdiv(tot, 256), 256, 0, st>>>(frames, F, H, W, fstride, rstride, d_crops, N, S, mean, scale, 3,
                                                          (float*)out);
    else if (bf16)
        k_blob<__bf16, 1><<<cdiv(tot, 256), 256, 0, st>>>(frames, F, H, W, fstride, rstride, d_crops, N, S, mean, scale,
                                                           Cp, (__bf16*)out);
    else
        k_blob<float, 1><<<cdiv(tot, 256), 256, 0, st>>>(frames, F, H, W, fstride, rstride, d_crops, N, S, mean, scale, Cp,
                                                          (float*)out);
}

}  // namespace vtf

using namespace vtf;

extern "C" int vtf_blob_from_crops(const uint8_t* d_frames, int F, int H, int W, int64_t frame_stride, int64_t row_stride,
                                   const int32_t* d_crops, int64_t N, int S, float mean, float scale, float* d_out,
                                   void* hip_stream) {
    return guarded_on(stream_device((hipStream_t)hip_stream), [&] {
        VTF_CHECK(N >= 0 && S > 0, VTF_E_ARG, "bad argument");
        if (N == 0) return;
        VTF_CHECK(d_frames && d_crops && d_out, VTF_E_ARG, "null argument");
        launch_blob(d_frames, F, H, W, frame_stride, row_stride, d_crops, N, S, mean, scale, 0, 3, false, d_out,
                    (hipStream_t)hip_stream);
        VTF_HIP(hipGetLastError());
    });
}

// Hash-based near-duplicate removal on gfx950 (src/videotofaces/dupes.py:11-59).
//
//   k_ahash: dupes.ahash (dupes.py:11-15) for every face crop straight from the frames in HBM,
//     one wave per crop, one lane per pixel of the 8x8 thumbnail:
//       cv2.cvtColor(BGR2GRAY): Y = (1868 B + 9617 G + 4899 R + 2^13) >> 14 (OpenCV fixed point);
//       cv2.resize(gray, (8, 8)) INTER_LINEAR (11-bit coefficients, blob.hpp lin_coef; OpenCV
//       switches to INTER_AREA for an exact 2x downscale, i.e. 16x16 crops);
//       tiny > np.mean(tiny)  <=>  64 * tiny > sum(tiny) (exact integers) -> wave ballot = the
//       64-bit hash, bit k = thumbnail pixel k in row-major order (diff.flatten()).
//   k_hamming_lower: remove_dupes_overall('hash') (dupes.py:55-65): for every face i, min and
//     first argmin over j < i of popcount(h_i ^ h_j) -- the reference's O(N^2) Python-lambda
//     pairwise_distances, with its strict-lower-triangle mask (row 0 -> 10000 at index 0).
// cv2 is absent in this image: the cvtColor/resize restatement is parity-UNPINNED (see
// DESIGN.md); the Hamming dedupe is pinned by the reference's own remove_dupes_overall.
#include <cstring>
#include <vector>

#include "blob.hpp"
#include "boxes.hpp"
#include "common.hpp"

namespace vtf {

__device__ inline int gray_at(const uint8_t* p) {
    return ((int)p[0] * 1868 + (int)p[1] * 9617 + (int)p[2] * 4899 + (1 << 13)) >> 14;
}

__global__ __launch_bounds__(64) void k_ahash(const uint8_t* __restrict__ frames, int H, int W, int64_t fstride,
                                              int64_t rstride, const int32_t* __restrict__ crops, int64_t N,
                                              uint64_t* __restrict__ out) {
    const int64_t n = blockIdx.x;
    const int lane = threadIdx.x;
    const int32_t* c = crops + n * 5;
    int x1 = max(0, min(c[1], W)), x2 = max(x1, min(c[3], W));
    int y1 = max(0, min(c[2], H)), y2 = max(y1, min(c[4], H));
    const int w = x2 - x1, h = y2 - y1;
    const uint8_t* base = frames + (int64_t)c[0] * fstride + (int64_t)y1 * rstride + (int64_t)x1 * 3;
    const int dx = lane & 7, dy = lane >> 3;
    int v = 0;
    if (w > 0 && h > 0) {
        if (w == 16 && h == 16) {
            // INTER_AREA fast path (resizeAreaFast, 2x2 average with rounding)
            const uint8_t* r0 = base + (int64_t)(2 * dy) * rstride + 2 * dx * 3;
            const uint8_t* r1 = r0 + rstride;
            v = (gray_at(r0) + gray_at(r0 + 3) + gray_at(r1) + gray_at(r1 + 3) + 2) >> 2;
        } else {
            int sx0, sx1, a0, a1, sy0, sy1, b0, b1;
            bool ex, ey;
            lin_coef(dx, w, 8, sx0, sx1, a0, a1, ex);
            lin_coef(dy, h, 8, sy0, sy1, b0, b1, ey);
            (void)ey;
            const uint8_t* r0 = base + (int64_t)sy0 * rstride;
            const uint8_t* r1 = base + (int64_t)sy1 * rstride;
            const int g00 = gray_at(r0 + sx0 * 3), g01 = gray_at(r0 + sx1 * 3);
            const int g10 = gray_at(r1 + sx0 * 3), g11 = gray_at(r1 + sx1 * 3);
            const int h0 = ex ? g00 * 2048 : g00 * a0 + g01 * a1;
            const int h1 = ex ? g10 * 2048 : g10 * a0 + g11 * a1;
            v = min(255, max(0, ((((h0 >> 4) * b0) >> 16) + (((h1 >> 4) * b1) >> 16) + 2) >> 2));
        }
    }
    int sum = v;
    for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off);
    const uint64_t bits = __ballot(64 * v > sum);
    if (lane == 0) out[n] = bits;
}

// one thread per row i, hashes of j < i streamed through LDS in 1024-entry tiles
__global__ __launch_bounds__(256) void k_hamming_lower(const uint64_t* __restrict__ hs, int64_t N,
                                                       int32_t* __restrict__ mn, int64_t* __restrict__ arg) {
    __shared__ uint64_t tile[1024];
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int64_t bend = ((int64_t)blockIdx.x + 1) * blockDim.x;
    const int64_t last = bend < N ? bend : N;  // rows of this block are < last
    const uint64_t hi = i < N ? hs[i] : 0ull;
    int best = 1 << 30;
    int64_t barg = 0;
    for (int64_t j0 = 0; j0 < last - 1; j0 += 1024) {
        __syncthreads();
        for (int t = threadIdx.x; t < 1024; t += blockDim.x)
            if (j0 + t < N) tile[t] = hs[j0 + t];
        __syncthreads();
        int64_t jend = i - j0 < 1024 ? i - j0 : 1024;
        if (jend > N - j0) jend = N - j0;
        for (int64_t t = 0; t < jend; t++) {
            const int d = __popcll(hi ^ tile[t]);
            if (d < best) {
                best = d;
                barg = j0 + t;
            }
        }
    }
    if (i < N) {
        if (i == 0) {
            mn[i] = 10000;  // every entry of row 0 is masked: D[0,0] + 10000 (dupes.py:62)
            arg[i] = 0;
        } else {
            mn[i] = best;
            arg[i] = barg;
        }
    }
}

}  // namespace vtf

using namespace vtf;

extern "C" {

int vtf_ahash_crops(const uint8_t* d_frames, int F, int H, int W, int64_t frame_stride, int64_t row_stride,
                    const int32_t* crops, int64_t N, uint64_t* out_hashes, void* hip_stream) {
    return guarded_on(stream_device((hipStream_t)hip_stream), [&] {
        VTF_CHECK(N >= 0 && H > 0 && W > 0, VTF_E_ARG, "bad argument");
        if (N == 0) return;
        VTF_CHECK(d_frames && crops && out_hashes, VTF_E_ARG, "null argument");
        check_crops_host(crops, N, F, H, W);
        hipStream_t st = (hipStream_t)hip_stream;
        int32_t* dc = nullptr;
        uint64_t* dh = nullptr;
        VTF_HIP(hipMallocAsync((void**)&dc, N * 20, st));
        VTF_HIP(hipMallocAsync((void**)&dh, N * 8, st));
        VTF_HIP(hipMemcpyAsync(dc, crops, N * 20, hipMemcpyHostToDevice, st));
        k_ahash<<<(unsigned)N, 64, 0, st>>>(d_frames, H, W, frame_stride, row_stride, dc, N, dh);
        VTF_HIP(hipMemcpyAsync(out_hashes, dh, N * 8, hipMemcpyDeviceToHost, st));
        VTF_HIP(hipFreeAsync(dc, st));
        VTF_HIP(hipFreeAsync(dh, st));
        VTF_HIP(hipStreamSynchronize(st));
    });
}

int vtf_hamming_dedupe(const uint64_t* d_hashes, int64_t N, int32_t* d_min, int64_t* d_arg, void* hip_stream) {
    return guarded_on(stream_device((hipStream_t)hip_stream), [&] {
        VTF_CHECK(N >= 0, VTF_E_ARG, "bad argument");
        if (N == 0) return;
        VTF_CHECK(d_hashes && d_min && d_arg, VTF_E_ARG, "null argument");
        hipStream_t st = (hipStream_t)hip_stream;
        k_hamming_lower<<<cdiv(N, 256), 256, 0, st>>>(d_hashes, N, d_min, d_arg);
        VTF_HIP(hipGetLastError());
    });
}

}  // extern "C"

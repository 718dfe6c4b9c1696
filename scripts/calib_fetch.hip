// FETCH_SIZE calibration on gfx950 for the access widths k_pnet's PR launch uses.
// MI355X_MICROARCH.md calibrates FETCH_SIZE only for 16-B-per-lane streaming reads (it reports
// half the bytes there) and leaves other widths uncalibrated.  The PR launch reads its
// precomputed split levels as 12-B pixels (one global_load_dwordx3 per lane), so its
// "x 2"-corrected fetch in profiles/pnet_traffic.json rests on an unmeasured factor.  Each kernel
// below reads a known number of distinct bytes once (buffer 768 MiB, past the 256 MiB Infinity
// Cache); tile12 reads the PR launch's level window pattern (42 x 44 pixels per 32 x 32 tile, two
// halves of 22 rows), whose bytes are counted exactly on the host.
// Build: hipcc -O3 --offload-arch=gfx950 scripts/calib_fetch.hip -o gpurun_out/calib_fetch
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <cstdlib>

#define CK(x)                                                                           \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

__global__ void rd16(const uint4* __restrict__ p, int64_t n, uint32_t* sink) {
    uint32_t a = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const uint4 v = p[i];
        a ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (a == 0x9e3779b9u) sink[threadIdx.x] = a;  // never true for the zero-filled buffer
}

__global__ void rd12(const uint3* __restrict__ p, int64_t n, uint32_t* sink) {
    uint32_t a = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) {
        const uint3 v = p[i];
        a ^= v.x ^ v.y ^ v.z;
    }
    if (a == 0x9e3779b9u) sink[threadIdx.x] = a;
}

__global__ void rd4(const uint32_t* __restrict__ p, int64_t n, uint32_t* sink) {
    uint32_t a = 0;
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n; i += (int64_t)gridDim.x * 256) a ^= p[i];
    if (a == 0x9e3779b9u) sink[threadIdx.x] = a;
}

// one workgroup per 32 x 32 tile of an lh x lw level of 12-B pixels: rows [20 h, 20 h + 22) of the
// tile's 42-column window for h = 0, 1 (k_pnet's PR fill: lanes along the row, 6 rows per pass)
constexpr int PW = 42, HR = 22;
__global__ void tile12(const uint3* __restrict__ p, int lh, int lw, int tiles_x, uint32_t* sink) {
    const int tx = blockIdx.x % tiles_x, ty = blockIdx.x / tiles_x;
    const int t = threadIdx.x, fq = t % PW, fr0 = t < 6 * PW ? t / PW : HR;
    const int lx = 32 * tx + fq;
    uint32_t a = 0;
    for (int h = 0; h < 2; h++)
        for (int j = 0; j < 4; j++) {
            const int r = fr0 + 6 * j, ly = 32 * ty + 20 * h + r;
            if (r < HR && lx < lw && ly < lh) {
                const uint3 v = p[(int64_t)ly * lw + lx];
                a ^= v.x ^ v.y ^ v.z;
            }
        }
    if (a == 0x9e3779b9u) sink[threadIdx.x] = a;
}

int main() {
    const int64_t B = 3ll << 28;  // 768 MiB
    char* buf;
    uint32_t* sink;
    CK(hipMalloc(&buf, B));
    CK(hipMalloc(&sink, 1024));
    CK(hipMemset(buf, 0, B));
    CK(hipDeviceSynchronize());
    const int grid = 256 * 16;
    for (int rep = 0; rep < 3; rep++) {
        rd16<<<grid, 256>>>((const uint4*)buf, B / 16, sink);
        rd12<<<grid, 256>>>((const uint3*)buf, B / 12, sink);
        rd4<<<grid, 256>>>((const uint32_t*)buf, B / 4, sink);
    }
    // a level of 12-B pixels: 4096 x 8192 = 402.7 MB
    const int lh = 8192, lw = 4096, tx = (lw + 31) / 32, ty = (lh + 31) / 32;
    int64_t win = 0;  // bytes the window reads (distinct per tile, overlapping between tiles)
    for (int y = 0; y < ty; y++)
        for (int x = 0; x < tx; x++) {
            const int cw = std::min(PW, lw - 32 * x);
            for (int h = 0; h < 2; h++) {
                const int rows = std::max(0, std::min(HR, lh - (32 * y + 20 * h)));
                win += (int64_t)rows * cw * 12;
            }
        }
    for (int rep = 0; rep < 3; rep++) tile12<<<tx * ty, 256>>>((const uint3*)buf, lh, lw, tx, sink);
    CK(hipGetLastError());
    CK(hipDeviceSynchronize());
    std::printf("rd16 / rd12 / rd4: %lld distinct bytes each per launch\n", (long long)B);
    std::printf("tile12: level %lld distinct bytes, window reads %lld bytes per launch (%.3f x)\n",
                (long long)lh * lw * 12, (long long)win, (double)win / ((double)lh * lw * 12));
    CK(hipFree(buf));
    CK(hipFree(sink));
    return 0;
}

// Probe: issue cycles per MFMA on one SIMD (one wave, 4 independent accumulators) for the
// fp16 16x16x16 and 16x16x32 forms and the fp32 16x16x4 form.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(4))) _Float16 f16x4;
typedef __attribute__((ext_vector_type(8))) _Float16 f16x8;
template <int V>
__global__ void k(float* out, long long* cyc) {
    f32x4 c[4] = {};
    f16x4 a4 = {(_Float16)threadIdx.x, 1, 2, 3};
    f16x8 a8 = {(_Float16)threadIdx.x, 1, 2, 3, 4, 5, 6, 7};
    float af = threadIdx.x;
    long long t0 = clock64();
    for (int it = 0; it < 256; it++) {
#pragma unroll
        for (int q = 0; q < 4; q++) {
            if (V == 0) c[q] = __builtin_amdgcn_mfma_f32_16x16x16f16(a4, a4, c[q], 0, 0, 0);
            if (V == 1) c[q] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a8, a8, c[q], 0, 0, 0);
            if (V == 2) c[q] = __builtin_amdgcn_mfma_f32_16x16x4f32(af, af, c[q], 0, 0, 0);
        }
    }
    long long t1 = clock64();
    float s = 0;
    for (int q = 0; q < 4; q++) s += c[q][0] + c[q][1] + c[q][2] + c[q][3];
    out[threadIdx.x] = s;
    if (threadIdx.x == 0) *cyc = t1 - t0;
}
int main() {
    float* d;
    long long* c;
    (void)hipMalloc(&d, 256 * 4);
    (void)hipMalloc(&c, 8);
    const char* nm[3] = {"16x16x16_f16", "16x16x32_f16", "16x16x4_f32"};
    for (int v = 0; v < 3; v++) {
        for (int rep = 0; rep < 2; rep++) {
            if (v == 0) k<0><<<1, 64>>>(d, c);
            if (v == 1) k<1><<<1, 64>>>(d, c);
            if (v == 2) k<2><<<1, 64>>>(d, c);
            long long h;
            (void)hipMemcpy(&h, c, 8, hipMemcpyDeviceToHost);
            if (rep) printf("%s: %.2f cycles per MFMA\n", nm[v], h / 1024.0);
        }
    }
    return 0;
}

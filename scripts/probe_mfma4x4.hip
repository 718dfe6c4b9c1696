// Probe: operand / result lane layout of v_mfma_f32_4x4x1_16b_f32 on gfx950.
// A[b][i] = 100*b + i (lane supplies a), B[b][j] = j + 1 (lane supplies b); prints which
// (block, row, col) each (lane, reg) of D holds, decoded from D = A*B.
#include <hip/hip_runtime.h>
#include <cstdio>
typedef __attribute__((ext_vector_type(4))) float f32x4;
__global__ void k(float* out) {
    int l = threadIdx.x;
    float a = (float)(1000 * (l / 4) + (l % 4));  // guess: lane = 4*block + i
    float b = (float)(1 << (l % 4));              // guess: lane = 4*block + j
    if (l / 4 == 3) b *= 16.f;                    // mark block 3 of B
    f32x4 c = {0.f, 0.f, 0.f, 0.f};
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; r++) out[l * 4 + r] = c[r];
}
int main() {
    float* d;
    hipMalloc(&d, 256 * 4);
    k<<<1, 64>>>(d);
    float h[256];
    hipMemcpy(h, d, 1024, hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; l++) {
        printf("lane %2d:", l);
        for (int r = 0; r < 4; r++) printf(" %9.0f", h[l * 4 + r]);
        printf("\n");
    }
    return 0;
}

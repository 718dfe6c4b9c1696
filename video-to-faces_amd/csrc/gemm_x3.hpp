#pragma once
#include "common.hpp"

namespace vtf {

// "Split pairs" (SP) operand layout of the fp32-grade fp16 GEMM: a row of K fp32 values
// (K % 8 == 0) is stored as K/8 chunks of 32 bytes, chunk j = [x0 of elements 8j..8j+7 (8 x fp16)]
// [x1 of the same 8 (8 x fp16)], x = x0 + x1 * 2^-11 with x0 = fp16(x), x1 = fp16((x - x0) * 2^11).
// Same bytes as fp32 (4 per element); a 16-byte piece is one MFMA fragment row of one plane.
// Valid for |x| < 2^14 (producers raise *ovf otherwise).
struct GemmX3Params {
    const void* a;       // SP [M][K]
    const void* b;       // SP [N][K] (weights, split once on the host)
    void* out;           // fp32 [M][ldo], or SP [M][N] when out_sp
    const float* bias;   // [N] or null
    const float* res;    // fp32 [M][ldr] or null: added after the bias
    int* ovf;            // out_sp: set to 1 when an output leaves the fp16 range (or is NaN)
    int64_t M;
    int N, K, ldo, ldr;
    int gelu;            // exact erf GELU after bias / residual (ViT MLP, vit.py:37)
    int out_sp;
    // set by launch_gemm_x3: tile grid, XCD-aware order, whole tiles vs split-K tail tiles
    int gx, gy, group_m;
    int dp_tiles;        // work items < dp_tiles are whole tiles
    int tail_split;      // the remaining tiles run as tail_split K slices each
    float* ws;           // tail partial sums [tail tiles][tail_split][BM * BN] (k_gemm_x3_tail reduces)
    int64_t lda, ldb;    // row strides of a / b in bytes (0: K * 4, dense)
};

// C = A B^T (+ bias) (+ res) (GELU): K % 32 == 0, N % 8 == 0
void launch_gemm_x3(const GemmX3Params& p, hipStream_t st);
// fp32 rows [rows][K] (row stride ld floats) -> SP [rows][K]; |x| >= 2^14 or NaN sets *ovf
void launch_split_rows(const float* x, int64_t rows, int K, int64_t ld, void* out, int* ovf, hipStream_t st);
// host-side split of fp32 rows into SP (weights); returns false when a value leaves the fp16 range
bool split_rows_host(const float* x, int64_t rows, int K, uint16_t* out);

// SP store of 4 consecutive elements e0..e0+3 (e0 % 4 == 0) of a row: 8-byte x0 and x1 pieces
__device__ inline void sp_store4(void* row, int e0, float a, float b, float c, float d, bool& bad) {
    typedef __attribute__((ext_vector_type(4))) _Float16 h4;
    h4 x0, x1;
    const float v[4] = {a, b, c, d};
#pragma unroll
    for (int e = 0; e < 4; e++) {
        x0[e] = (_Float16)v[e];
        x1[e] = (_Float16)((v[e] - (float)x0[e]) * 2048.f);
        bad |= !(fabsf(v[e]) < 16384.f);
    }
    char* base = (char*)row + (e0 >> 3) * 32 + (e0 & 4) * 2;
    *(h4*)base = x0;
    *(h4*)(base + 16) = x1;
}

}  // namespace vtf

// Device helpers shared by the conv kernels (conv.hip, conv_dma.hip): element conversions and
// the fused conv epilogue (bias / BN / scale / residual / activation / layout).
#pragma once
#include "common.hpp"
#include "conv.hpp"
#include "gemm_x3.hpp"

namespace vtf {

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;

template <typename T>
struct VecT;
template <>
struct VecT<float> {
    typedef f32x4 type;
    static constexpr int V = 4;
};
template <>
struct VecT<__bf16> {
    typedef bf16x8 type;
    static constexpr int V = 8;
};

__device__ inline float to_f(float v) { return v; }
__device__ inline float to_f(__bf16 v) { return (float)v; }
template <typename T>
__device__ inline T from_f(float v);
template <>
__device__ inline float from_f<float>(float v) { return v; }
template <>
__device__ inline __bf16 from_f<__bf16>(float v) { return (__bf16)v; }

// residual element index of output (m, c): same layout as the output, or the half-resolution
// map of the FPN top-down add (res_up2)
__device__ inline int64_t res_index(const ConvParams& p, int64_t m, int c) {
    if (!p.res_up2) return m * p.res_cstride + c;
    const int ow = (int)(m % p.OW);
    const int64_t t = m / p.OW;
    const int oh = (int)(t % p.OH);
    const int64_t n = t / p.OH;
    return ((n * (p.OH >> 1) + (oh >> 1)) * (p.OW >> 1) + (ow >> 1)) * p.res_cstride + c;
}

// fused epilogue of one output element (bias / BN / scale / residual / activation / layout);
// rv = the residual element (loaded by the caller: a workgroup's residual loads are issued
// together, not one round trip per output behind the previous store)
template <typename T>
__device__ inline void conv_epilogue(const ConvParams& p, int64_t m, int c, float v, float bias, float al, float be,
                                     float pr, float rv) {
    T* __restrict__ out = (T*)p.out;
    if (p.bias) v = v + bias;
    if (p.alpha) v = fmaf(v, al, be);
    if (p.scale != 1.f) v = v * p.scale;
    if (p.res && !p.res_post) v = v + rv;
    if (p.relu) v = fmaxf(v, 0.f);
    if (p.leaky) v = v > 0.f ? v : v * p.slope;
    if (p.prelu) v = v > 0.f ? v : pr * v;
    if (p.gelu) v = 0.5f * v * (1.0f + erff(v * 0.70710678118654752f));
    if (p.res && p.res_post) v = v + rv;
    if (p.up2) {
        int ow = (int)(m % p.OW);
        int64_t t = m / p.OW;
        int oh = (int)(t % p.OH);
        int64_t n = t / p.OH;
        int64_t o = ((n * 2 * p.OH + 2 * oh) * 2 * p.OW + 2 * ow) * p.out_cstride + p.out_coff + c;
        int64_t rs = (int64_t)2 * p.OW * p.out_cstride;
        T tv = from_f<T>(v);
        out[o] = tv;
        out[o + p.out_cstride] = tv;
        out[o + rs] = tv;
        out[o + rs + p.out_cstride] = tv;
    } else if (p.out_f32) {
        ((float*)p.out)[m * p.out_cstride + p.out_coff + c] = v;
    } else if (p.n_split && c >= p.n_split) {
        ((T*)p.out2)[m * p.out2_cstride + p.out2_coff + (c - p.n_split)] = from_f<T>(v);
    } else {
        out[m * p.out_cstride + p.out_coff + c] = from_f<T>(v);
    }
}

// "Split-triple" (S3) layout of the bf16x3 mode (conv_dma MODE 2): a row of C fp32 values
// (C % 8 == 0) is stored as C/8 chunks of 48 bytes, chunk j = [b0 | b1 | b2] of elements
// 8j..8j+7 (8 bf16 each) with b0 = bf16(x), b1 = bf16(x - b0), b2 = x - b0 - b1 (exact in bf16:
// x has 24 significant bits, b0 and b1 take 8 each).  x = (b0 + b1) + b2 exactly, so one S3
// tensor is both the next conv's operand and an exact fp32 residual; the bf16 exponent range is
// fp32's (no range guard, unlike the fp16 split pairs).
__device__ inline void s3_store8(char* q, const float (&v)[8]) {
    bf16x8 h0, h1, h2;
#pragma unroll
    for (int e = 0; e < 8; e++) {
        const __bf16 a = (__bf16)v[e];
        const float r1 = v[e] - (float)a;
        const __bf16 b = (__bf16)r1;
        h0[e] = a;
        h1[e] = b;
        h2[e] = (__bf16)(r1 - (float)b);
    }
    *(bf16x8*)q = h0;
    *(bf16x8*)(q + 16) = h1;
    *(bf16x8*)(q + 32) = h2;
}
__device__ inline void s3_load8(const char* q, float (&v)[8]) {
    const bf16x8 h0 = *(const bf16x8*)q, h1 = *(const bf16x8*)(q + 16), h2 = *(const bf16x8*)(q + 32);
#pragma unroll
    for (int e = 0; e < 8; e++) v[e] = ((float)h0[e] + (float)h1[e]) + (float)h2[e];
}

// 8 consecutive output channels c0..c0+7 of row m (c0 % 8 == 0, channel strides / offsets
// multiples of 8): the same element math as conv_epilogue with 16/32-byte loads and stores
template <typename T>
__device__ inline void conv_epilogue8(const ConvParams& p, int64_t m, int c0, float (&v)[8], const float (&b8)[8],
                                      const float (&al8)[8], const float (&be8)[8], const float (&pr8)[8],
                                      bool* bad = nullptr) {
    typedef __attribute__((ext_vector_type(8))) T t8;
    float rv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if (p.res && p.s3) {
        s3_load8((const char*)p.res + (res_index(p, m, c0) >> 3) * 48, rv);
    } else if (p.res) {
        const t8 r = *(const t8*)((const T*)p.res + res_index(p, m, c0));
#pragma unroll
        for (int e = 0; e < 8; e++) rv[e] = to_f(r[e]);
    }
    t8 o;
#pragma unroll
    for (int e = 0; e < 8; e++) {
        float x = v[e];
        if (p.bias) x = x + b8[e];
        if (p.alpha) x = fmaf(x, al8[e], be8[e]);
        if (p.scale != 1.f) x = x * p.scale;
        if (p.res && !p.res_post) x = x + rv[e];
        if (p.relu) x = fmaxf(x, 0.f);
        if (p.leaky) x = x > 0.f ? x : x * p.slope;
        if (p.prelu) x = x > 0.f ? x : pr8[e] * x;
        if (p.gelu) x = 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
        if (p.res && p.res_post) x = x + rv[e];
        v[e] = x;
        o[e] = from_f<T>(x);
    }
    if (p.up2 && p.s3 && !p.out_f32) {
        const int ow = (int)(m % p.OW);
        const int64_t t = m / p.OW;
        const int oh = (int)(t % p.OH);
        const int64_t n = t / p.OH;
        const int64_t a = ((n * 2 * p.OH + 2 * oh) * 2 * p.OW + 2 * ow) * p.out_cstride + p.out_coff + c0;
        const int64_t rs = (int64_t)2 * p.OW * p.out_cstride;
        char* out = (char*)p.out;
        s3_store8(out + (a >> 3) * 48, v);
        s3_store8(out + ((a + p.out_cstride) >> 3) * 48, v);
        s3_store8(out + ((a + rs) >> 3) * 48, v);
        s3_store8(out + ((a + rs + p.out_cstride) >> 3) * 48, v);
    } else if (p.up2) {
        const int ow = (int)(m % p.OW);
        const int64_t t = m / p.OW;
        const int oh = (int)(t % p.OH);
        const int64_t n = t / p.OH;
        T* out = (T*)p.out;
        const int64_t a = ((n * 2 * p.OH + 2 * oh) * 2 * p.OW + 2 * ow) * p.out_cstride + p.out_coff + c0;
        const int64_t rs = (int64_t)2 * p.OW * p.out_cstride;
        *(t8*)(out + a) = o;
        *(t8*)(out + a + p.out_cstride) = o;
        *(t8*)(out + a + rs) = o;
        *(t8*)(out + a + rs + p.out_cstride) = o;
    } else if (p.out_sp) {
        // split-pair layout (gemm_x3.hpp) for a split-fp16 consumer; row stride out_cstride * 4 bytes
        bool b = false;
        char* row = (char*)p.out + m * (int64_t)p.out_cstride * 4;
        sp_store4(row, p.out_coff + c0, v[0], v[1], v[2], v[3], b);
        sp_store4(row, p.out_coff + c0 + 4, v[4], v[5], v[6], v[7], b);
        if (bad) *bad |= b;
    } else if (p.out_f32) {
        float* out = (float*)p.out + m * p.out_cstride + p.out_coff + c0;
        *(f32x4*)out = f32x4{v[0], v[1], v[2], v[3]};
        *(f32x4*)(out + 4) = f32x4{v[4], v[5], v[6], v[7]};
    } else if (p.s3) {
        s3_store8((char*)p.out + ((m * p.out_cstride + p.out_coff + c0) >> 3) * 48, v);
    } else if (p.n_split && c0 >= p.n_split) {
        *(t8*)((T*)p.out2 + m * p.out2_cstride + p.out2_coff + (c0 - p.n_split)) = o;
    } else {
        *(t8*)((T*)p.out + m * p.out_cstride + p.out_coff + c0) = o;
    }
}

}  // namespace vtf

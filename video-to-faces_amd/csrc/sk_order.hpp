// Float32 summation orders of the reference's CPU libraries (numpy 2.2 einsum, OpenBLAS
// SKYLAKEX level-3 drivers), measured by absorption probes in the survey container
// (scripts/sklearn_order.py, scripts/sklearn_cosine_order.py) and shared by the grouping
// kernels that must reproduce sklearn's bits (kmeans.hip, grouping.hip).
#pragma once
#include <hip/hip_runtime.h>

namespace vtf {

// row_norms(C, squared=True) = np.einsum('ij,ij->i', C, C): 4 SSE lanes over d mod 4; each
// 16-element step adds the products of elements 12..15, 8..11, 4..7, 0..3 in that order (mul,
// then add: no FMA in numpy's baseline); 4-element zero-padded tail steps; (l0 + l1) + (l2 + l3).
__device__ inline float np_einsum_sq(const float* __restrict__ c, int D) {
    float l[4] = {0.f, 0.f, 0.f, 0.f};
    int t = 0;
    for (; D - t >= 16; t += 16)
        for (int q = 3; q >= 0; q--)
#pragma unroll
            for (int u = 0; u < 4; u++) l[u] = __fadd_rn(__fmul_rn(c[t + 4 * q + u], c[t + 4 * q + u]), l[u]);
    for (; t < D; t += 4)
#pragma unroll
        for (int u = 0; u < 4; u++) {
            const float v = t + u < D ? c[t + u] : 0.f;
            l[u] = __fadd_rn(__fmul_rn(v, v), l[u]);
        }
    return __fadd_rn(__fadd_rn(l[0], l[1]), __fadd_rn(l[2], l[3]));
}

// OpenBLAS level-3 K blocking (GEMM_Q = 448 for SKYLAKEX sgemm): the length of the K block that
// starts with `rest` elements left.  gemm (driver/level3/level3.c) rounds the half of a
// remainder in (Q, 2Q) up to the unroll (16); syrk (level3_syrk.c) takes (rest + 1) / 2.
__host__ __device__ inline int blas_kblock(int rest, bool syrk) {
    if (rest >= 2 * 448) return 448;
    if (rest > 448) return syrk ? (rest + 1) / 2 : ((rest / 2 + 15) / 16) * 16;
    return rest;
}

}  // namespace vtf

/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may load this library; the product path never does.
 *
 * CPU restatement of the embedding dedupe of remove_dupes_overall('enc')
 * (src/videotofaces/dupes.py:60-65) in the bits of the reference's own libraries -- sklearn
 * 1.7.2 cosine_distances on numpy 2.2.6 and its bundled OpenBLAS 0.3.29 (SkylakeX kernels),
 * measured by absorption probes in the survey container (scripts/sklearn_cosine_order.py):
 *   norm_i  = sqrt(np.einsum('ij,ij->i', X, X))       numpy's SSE einsum order (4 lanes over
 *             d mod 4, each 16-element step adding elements 12..15, 8..11, 4..7, 0..3,
 *             multiply then add; (l0 + l1) + (l2 + l3)); 0 -> 1 (_handle_zeros_in_scale)
 *   xn      = X / norm                                (sklearn.preprocessing.normalize)
 *   G       = xn @ xn.T                               numpy matmul -> cblas_ssyrk: K in blocks
 *             (448, or both halves (r + 1) / 2 of a remainder r in (448, 896)), each block one
 *             fmaf chain from 0 in k order, C += block in order
 *   d       = clip(1 - G, 0, 2)                       (S *= -1; S += 1; np.clip)
 *   mins/inds over j < i (the + (1 - tri(k=-1)) * 10000 mask), first minimum; row 0 -> 10000, 0
 *
 * Build: oracle/Makefile (gcc -O2 -mfma -ffp-contract=off: fmaf is the one fused operation).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static float einsum_sq(const float* c, int D) {
    float l[4] = {0.f, 0.f, 0.f, 0.f};
    int t = 0;
    for (; D - t >= 16; t += 16)
        for (int q = 3; q >= 0; q--)
            for (int u = 0; u < 4; u++) {
                float p = c[t + 4 * q + u] * c[t + 4 * q + u];
                l[u] = p + l[u];
            }
    for (; t < D; t += 4)
        for (int u = 0; u < 4; u++) {
            float v = t + u < D ? c[t + u] : 0.f;
            float p = v * v;
            l[u] = p + l[u];
        }
    float a = l[0] + l[1], b = l[2] + l[3];
    return a + b;
}

static int kblock(int rest, int syrk) {
    if (rest >= 2 * 448) return 448;
    if (rest > 448) return syrk ? (rest + 1) / 2 : ((rest / 2 + 15) / 16) * 16;
    return rest;
}

/* sklearn normalize(X) in place into xn (row-major N x D) */
void ora_normalize(const float* X, int64_t N, int64_t D, float* xn) {
    for (int64_t i = 0; i < N; i++) {
        float n = sqrtf(einsum_sq(X + i * D, (int)D));
        if (n == 0.f) n = 1.f;
        for (int64_t k = 0; k < D; k++) xn[i * D + k] = X[i * D + k] / n;
    }
}

/* mins[i], inds[i] of the masked cosine-distance row i (dupes.py:60-65); rows in parallel
   (OpenMP), each row's arithmetic sequential as above */
void ora_cos_dedupe(const float* X, int64_t N, int64_t D, float* mins, int64_t* inds) {
    float* xn = (float*)malloc(sizeof(float) * (size_t)(N * D));
    float* xt = (float*)malloc(sizeof(float) * (size_t)(N * D)); /* k-major copy: xt[k][j] */
    ora_normalize(X, N, D, xn);
    for (int64_t i = 0; i < N; i++)
        for (int64_t k = 0; k < D; k++) xt[k * N + i] = xn[i * D + k];
#pragma omp parallel
    {
        float* tot = (float*)malloc(sizeof(float) * (size_t)(N > 0 ? N : 1));
        float* acc = (float*)malloc(sizeof(float) * (size_t)(N > 0 ? N : 1));
#pragma omp for schedule(dynamic, 16)
        for (int64_t i = 0; i < N; i++) {
            mins[i] = 10000.f;
            inds[i] = 0;
            if (i == 0) continue;
            for (int64_t j = 0; j < i; j++) tot[j] = 0.f;
            for (int64_t k0 = 0; k0 < D;) {
                int64_t k1 = k0 + kblock((int)(D - k0), 1);
                for (int64_t j = 0; j < i; j++) acc[j] = 0.f;
                for (int64_t k = k0; k < k1; k++) {
                    const float a = xn[i * D + k];
                    const float* b = xt + k * N;
                    for (int64_t j = 0; j < i; j++) acc[j] = fmaf(a, b[j], acc[j]);
                }
                for (int64_t j = 0; j < i; j++) tot[j] = tot[j] + acc[j];
                k0 = k1;
            }
            float best = INFINITY;
            int64_t bj = 0;
            for (int64_t j = 0; j < i; j++) {
                float d = 1.0f - tot[j];
                d = d < 0.f ? 0.f : (d > 2.f ? 2.f : d);
                if (d < best) {
                    best = d;
                    bj = j;
                }
            }
            mins[i] = best;
            inds[i] = bj;
        }
        free(tot);
        free(acc);
    }
    free(xn);
    free(xt);
}

/* the full cosine_distances(X) matrix (N x N, diagonal 0) in the same bits */
void ora_cos_distances(const float* X, int64_t N, int64_t D, float* out) {
    float* xn = (float*)malloc(sizeof(float) * (size_t)(N * D));
    ora_normalize(X, N, D, xn);
    for (int64_t i = 0; i < N; i++)
        for (int64_t j = 0; j < N; j++) {
            float tot = 0.f;
            for (int64_t k0 = 0; k0 < D;) {
                int64_t k1 = k0 + kblock((int)(D - k0), 1);
                float acc = 0.f;
                for (int64_t k = k0; k < k1; k++) acc = fmaf(xn[i * D + k], xn[j * D + k], acc);
                tot = tot + acc;
                k0 = k1;
            }
            float d = 1.0f - tot;
            out[i * N + j] = i == j ? 0.f : (d < 0.f ? 0.f : (d > 2.f ? 2.f : d));
        }
    free(xn);
}

/* ---- classify (grouping.py:50-53): cosine_distances(X, R) in the reference's bits ----
 * X_n @ R_n.T is numpy matmul on two distinct buffers -> cblas_sgemm(RowMajor, NoTrans, Trans,
 * N, C, D) = Fortran sgemm('T', 'N', C, N, D, 1, R_n, D, X_n, D, 0, G, C): the E-step's form
 * (kmeans.hip) with alpha 1 and beta 0.  mode 0: the library's choice (sk_gemm_mode); 1: the
 * blocked kernel (K blocks of gemm's rule, one fmaf chain per block from 0, G += block); 2: the
 * small-matrix kernel (16 lanes over d mod 16, one fmaf chain per lane, adjacent-pair lane tree,
 * halving tree on the C tile's edge block). */
static float gemm_dot(const float* a, const float* b, int D, int mode, int edge) {
    if (mode == 5) {
        /* sgemv_t's 4x2 kernel: 4 lanes over d mod 4, product then add; (l0 + l1) + (l2 + l3) */
        float l[4] = {0.f, 0.f, 0.f, 0.f};
        for (int k = 0; k < D; k++) {
            const float p = a[k] * b[k];
            l[k & 3] = l[k & 3] + p;
        }
        return (l[0] + l[1]) + (l[2] + l[3]);
    }
    if (mode == 3 || mode == 4 || mode == 6) {
        /* 3: sgemv_t's 4x4 kernel (numpy matmul with one side a single row): 8 lanes over d mod 8,
         *    one fmaf chain per lane; (l_u + l_{u+4}), then (a0 + a1) + (a2 + a3).
         * 6: sgemv_t's 4x1 kernel: the same lanes and tree, product then add (no fma).
         * 4: sdot (a single row times a single row): 64 lanes over d mod 64 as 8 accumulators of
         *    8 lanes, combined (((c0 + c1) + (c2 + c3)) + (c4 + c5)) + (c6 + c7), then the 8
         *    lanes as in 3.  (Probed for D % 64 == 0.) */
        const int L = mode == 4 ? 64 : 8;
        float l[64];
        for (int u = 0; u < L; u++) l[u] = 0.f;
        for (int k = 0; k < D; k++) {
            if (mode == 6) {
                const float p = a[k] * b[k];
                l[k % L] = l[k % L] + p;
            } else {
                l[k % L] = fmaf(a[k], b[k], l[k % L]);
            }
        }
        float v[8];
        for (int u = 0; u < 8; u++) v[u] = l[u];
        if (mode == 4)
            for (int u = 0; u < 8; u++) {
                const float c01 = l[u] + l[8 + u], c23 = l[16 + u] + l[24 + u];
                const float c45 = l[32 + u] + l[40 + u], c67 = l[48 + u] + l[56 + u];
                v[u] = ((c01 + c23) + c45) + c67;
            }
        const float a0 = v[0] + v[4], a1 = v[1] + v[5], a2 = v[2] + v[6], a3 = v[3] + v[7];
        return (a0 + a1) + (a2 + a3);
    }
    if (mode == 2) {
        float l[16];
        for (int u = 0; u < 16; u++) l[u] = 0.f;
        for (int k = 0; k < D; k++) l[k & 15] = fmaf(a[k], b[k], l[k & 15]);
        if (edge) {
            for (int w = 8; w >= 1; w >>= 1)
                for (int u = 0; u < w; u++) l[u] = l[u] + l[u + w];
        } else {
            for (int w = 1; w < 16; w <<= 1)
                for (int u = 0; u < 16; u += 2 * w) l[u] = l[u] + l[u + w];
        }
        return l[0];
    }
    float tot = 0.f;
    for (int k0 = 0; k0 < D;) {
        int k1 = k0 + kblock(D - k0, 0);
        float acc = 0.f;
        for (int k = k0; k < k1; k++) acc = fmaf(a[k], b[k], acc);
        tot = tot + acc;
        k0 = k1;
    }
    return tot;
}

int ora_sk_gemm_mode(int64_t N, int64_t C, int64_t D) {
    if (N == 1 && C == 1) return 4;
    if (N == 1 || C == 1) return 3;
    return ((double)N * C * D <= 1e6 && C * N <= 1200 && D >= 32) ? 2 : 1;
}

/* Which sgemv_t kernel computes output o of n (numpy's gemv calls: one output per row of the
 * many-row side).  OpenBLAS splits the outputs over its threads when m * n >= 460800 (m = D;
 * measured: 8 threads in the survey container, ranges of ceil(rest / threads left) outputs, at
 * least 4); in each range groups of 4 take the 4x4 kernel, then 2 the 4x2 and 1 the 4x1. */
int ora_gemv_kernel(int64_t o, int64_t n, int64_t D, int threads) {
    int64_t a = 0;
    int T = (double)n * D >= 460800.0 ? threads : 1;
    for (int t = 0; a < n; t++) {
        int64_t w = T - t > 1 ? (n - a + (T - t) - 1) / (T - t) : n - a;
        if (w < 4) w = 4;
        if (w > n - a) w = n - a;
        if (o < a + w) {
            const int64_t r = o - a, q = w / 4 * 4;
            if (r < q) return 3;
            return (w & 2) && r < q + 2 ? 5 : 6;
        }
        a += w;
    }
    return 3;
}

void ora_cos_classify_dist(const float* X, int64_t N, const float* R, int64_t C, int64_t D, int mode, float* out) {
    float* xn = (float*)malloc(sizeof(float) * (size_t)(N * D));
    float* rn = (float*)malloc(sizeof(float) * (size_t)(C * D));
    ora_normalize(X, N, D, xn);
    ora_normalize(R, C, D, rn);
    if (mode == 0) mode = ora_sk_gemm_mode(N, C, D);
#pragma omp parallel for schedule(static)
    for (int64_t i = 0; i < N; i++)
        for (int64_t c = 0; c < C; c++) {
            const int edge = i >= N - N % 4 && c >= C - C % 4;
            int md = mode;
            if (mode == 3) md = C == 1 ? ora_gemv_kernel(i, N, D, 8) : ora_gemv_kernel(c, C, D, 8);
            float d = 1.0f - gemm_dot(xn + i * D, rn + c * D, (int)D, md, edge);
            out[i * C + c] = d < 0.f ? 0.f : (d > 2.f ? 2.f : d);
        }
    free(xn);
    free(rn);
}

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

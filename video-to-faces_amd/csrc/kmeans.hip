// Grouping on gfx950 (src/videotofaces/grouping.py:92-120 -> sklearn KMeans / silhouette /
// Calinski-Harabasz / Davies-Bouldin).  The Python mirror (videotofaces/kmeans.py) runs the
// scalar control flow of sklearn 1.7 (RandomState draws, searchsorted, convergence tests)
// on host numpy; every O(N*D) / O(N^2*D) pass is one of these kernels.
//
//   k_colstats     X.mean(axis=0), X - mean, np.var(X, axis=0): per-column sequential fp32
//                  sums in row order -- bit-identical to numpy's axis-0 reduction.
//   k_sqdist_rows  _euclidean_distances(X[ids], X, squared=True) for float32 X: the
//                  float64-upcast formula (-2 x.y + |x|^2 + |y|^2 in double, then float32,
//                  max 0; sklearn/metrics/pairwise.py:391-441,582-660).
//   k_estep        Lloyd E-step (_k_means_lloyd.pyx:_update_chunk_dense) in sklearn's bits:
//                  numpy's einsum order for |c|^2, OpenBLAS's sgemm orders for -2 x.c (see
//                  below), first strict minimum; counts label changes.
//   k_seg_*, k_msum_seq  M-step sums in sklearn's single-thread order (sequential fp32 per
//                  cluster and feature, rows in order) via a stable counting sort by label.
//   k_average      _average_centers (c *= 1/w) and _center_shift (4-way unrolled fp32).
//   k_pdist        full N x N euclidean matrix (pairwise_distances_chunked): float64 tile
//                  GEMM + norms, rounded to fp32, sqrt, zero diagonal.  Kept resident in HBM
//                  and reused for every k of a sweep.
//   k_silhouette   _silhouette_reduce + silhouette_samples per row (one wave per row).
//   k_csum/k_cdist cluster sums / |x|^2 / distance-to-centroid sums in float64 (CH, DB).
#include <cmath>
#include <vector>

#include "common.hpp"
#include "sk_order.hpp"

namespace vtf {

// ------------------------------------------------------------------ column statistics
__global__ void k_colstats(const float* __restrict__ X, int64_t N, int D, float* __restrict__ Xc,
                           float* __restrict__ mean, float* __restrict__ var) {
    int d = blockIdx.x * blockDim.x + threadIdx.x;
    if (d >= D) return;
    float acc = 0.f;
    for (int64_t i = 0; i < N; i++) acc += X[i * D + d];
    float m = acc / (float)N;
    float a2 = 0.f;
    for (int64_t i = 0; i < N; i++) {
        float x = X[i * D + d] - m;
        if (Xc) Xc[i * D + d] = x;
        a2 += x * x;
    }
    mean[d] = m;
    var[d] = a2 / (float)N;
}

// ------------------------------------------------------------------ wave helpers
__device__ inline double wave_sum_f64(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}
__device__ inline float wave_sum_f32(float v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
    return v;
}

// ------------------------------------------------------------------ k-means++ distance rows
// out[t][j] = max(0, f32((-2 * x_r.x_j + |x_r|^2) + |x_j|^2)), r = rows[t], all in double
template <int TMAX>
__global__ __launch_bounds__(256) void k_sqdist_rows(const float* __restrict__ X, int64_t N, int D,
                                                     const int64_t* __restrict__ rows, int T, float* __restrict__ out) {
    extern __shared__ float sR[];  // [T][D]
    for (int e = threadIdx.x; e < T * D; e += blockDim.x) sR[e] = X[rows[e / D] * D + (e % D)];
    __syncthreads();
    const int lane = threadIdx.x & 63;
    double rn[TMAX];
#pragma unroll
    for (int t = 0; t < TMAX; t++) {
        double s = 0.0;
        if (t < T)
            for (int d = lane; d < D; d += 64) s += (double)sR[t * D + d] * (double)sR[t * D + d];
        rn[t] = wave_sum_f64(s);
    }
    const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t j = wid; j < N; j += nw) {
        double dot[TMAX], yy = 0.0;
#pragma unroll
        for (int t = 0; t < TMAX; t++) dot[t] = 0.0;
        for (int d = lane; d < D; d += 64) {
            double y = (double)X[j * D + d];
            yy += y * y;
#pragma unroll
            for (int t = 0; t < TMAX; t++)
                if (t < T) dot[t] += (double)sR[t * D + d] * y;
        }
        yy = wave_sum_f64(yy);
#pragma unroll
        for (int t = 0; t < TMAX; t++) {
            if (t < T) {
                double s = wave_sum_f64(dot[t]);
                double dd = -2.0 * s;
                dd += rn[t];
                dd += yy;
                float f = (float)dd;
                if (lane == 0) out[(int64_t)t * N + j] = fmaxf(f, 0.f);
            }
        }
    }
}

// ------------------------------------------------------------------ Lloyd E-step, sklearn's bits
// _update_chunk_dense (_k_means_lloyd.pyx:168-215) on 256-row chunks: pd = |c|^2 (row_norms
// = np.einsum('ij,ij->i')), then scipy's sgemm adds -2 X C^T (_gemm RowMajor NoTrans/Trans ->
// Fortran sgemm('T', 'N', k, m, D, -2, C, D, X, D, 1, pd, k)), first strict minimum.  Both
// libraries' summation orders were measured bit for bit in the survey container (numpy 2.2
// with its SSE baseline einsum, scipy's OpenBLAS 0.3.28 SKYLAKEX kernels; probes by
// absorption -- 2^30, -2^30 and 1 at chosen positions -- then exact match on random data over
// D in {512, 768, 1024}, k 2..16, chunk rows 1..256; scripts/sklearn_order.py):
//   einsum  4 SSE lanes over d mod 4; each 16-element step adds the products of elements
//           12..15, 8..11, 4..7, 0..3 in that order (mul, then add: no FMA in the baseline);
//           4-element zero-padded tail steps; result (l0 + l1) + (l2 + l3).
//   sgemm, small-matrix kernel when m*k*D <= 1e6, k*m <= 1200 and D >= 32: 16 lanes over
//           d mod 16, sequential fma per lane; lanes summed as the adjacent-pair tree
//           ((l0+l1)+(l2+l3))+... except the C tile's edge block -- chunk row >= m - m%4 and
//           cluster >= k - k%4 -- which takes the halving tree (l_i + l_{i+8}, +4, +2, +1);
//           pd = pd - 2 s (one rounding: the x2 is exact).
//   sgemm, blocked kernel otherwise: D in K blocks (448, or the two halves of a remainder
//           between 448 and 896 rounded up to 16), sequential fma per block from 0, and
//           pd = pd - 2 acc after every block.
// (Exact for D % 16 == 0; other D follow the same rules without that verification.)
// (np_einsum_sq and the K blocking live in sk_order.hpp.)

__global__ void k_csq(const float* __restrict__ C, int k, int D, float* __restrict__ csq) {
    int j = blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= k) return;
    csq[j] = np_einsum_sq(C + (int64_t)j * D, D);
}

__host__ __device__ inline bool sk_small_gemm(int64_t m, int k, int D) {
    return (double)m * k * D <= 1e6 && (int64_t)k * m <= 1200 && D >= 32;
}

// one thread per (row, cluster): 16 rows x 16 clusters per block; X and C staged through LDS
// in 32-deep slices; the per-row argmin over the clusters at the end (first strict minimum)
constexpr int ES_R = 16, ES_C = 16, ES_K = 32;
__global__ __launch_bounds__(256) void k_estep(const float* __restrict__ X, int64_t N, int D,
                                               const float* __restrict__ C, const float* __restrict__ csq, int k,
                                               int32_t* __restrict__ labels, unsigned long long* __restrict__ changed) {
    __shared__ float sX[ES_R][ES_K + 1], sCt[ES_C][ES_K + 1];
    __shared__ float sD[ES_R][64 + 1];
    const int tid = threadIdx.x, r = tid >> 4, cj = tid & 15;
    const int64_t i0 = (int64_t)blockIdx.x * ES_R, i = i0 + r;
    // sklearn's 256-row chunk of this row: local row index and the chunk's row count
    const int64_t cs = (i0 / 256) * 256;
    const int m = (int)min<int64_t>(256, N - cs);
    const int il = (int)(i - cs);
    const bool small = sk_small_gemm(m, k, D);
    for (int j0 = 0; j0 < k; j0 += ES_C) {
        const int j = j0 + cj;
        float lane[16];
#pragma unroll
        for (int u = 0; u < 16; u++) lane[u] = 0.f;
        float acc = 0.f, pd = j < k ? csq[j] : 0.f;
        // K blocks of the blocked kernel (the small kernel ignores them)
        int kb_end = blas_kblock(D, false);
        for (int t0 = 0; t0 < D; t0 += ES_K) {
            for (int e = tid; e < ES_R * ES_K; e += 256) {
                const int rr = e / ES_K, tt = e % ES_K;
                sX[rr][tt] = (i0 + rr < N && t0 + tt < D) ? X[(i0 + rr) * D + t0 + tt] : 0.f;
                sCt[rr][tt] = (j0 + rr < k && t0 + tt < D) ? C[(int64_t)(j0 + rr) * D + t0 + tt] : 0.f;
            }
            __syncthreads();
            const int tn = min(ES_K, D - t0);
            if (small) {
#pragma unroll
                for (int tt = 0; tt < ES_K; tt++)
                    if (tt < tn) lane[(t0 + tt) & 15] = fmaf(sX[r][tt], sCt[cj][tt], lane[(t0 + tt) & 15]);
            } else {
                for (int tt = 0; tt < tn; tt++) {
                    acc = fmaf(sX[r][tt], sCt[cj][tt], acc);
                    if (t0 + tt + 1 == kb_end) {  // end of a K block: C += alpha * block
                        pd = fmaf(-2.f, acc, pd);
                        acc = 0.f;
                        kb_end += blas_kblock(D - kb_end, false);
                    }
                }
            }
            __syncthreads();
        }
        if (small) {
            float s;
            if (il >= m - m % 4 && j >= k - k % 4) {  // edge block of the C tile: halving tree
#pragma unroll
                for (int w = 8; w >= 1; w >>= 1)
#pragma unroll
                    for (int u = 0; u < w; u++) lane[u] = __fadd_rn(lane[u], lane[u + w]);
                s = lane[0];
            } else {  // adjacent pairs
#pragma unroll
                for (int w = 1; w < 16; w <<= 1)
#pragma unroll
                    for (int u = 0; u < 16; u += 2 * w) lane[u] = __fadd_rn(lane[u], lane[u + w]);
                s = lane[0];
            }
            pd = fmaf(-2.f, s, pd);
        }
        if (cj < 16) sD[r][j0 + cj < 64 ? (j0 + cj) : 64] = pd;
        __syncthreads();
        // (k <= 64: sD holds every cluster's distance for the rows of this block)
    }
    if (cj == 0 && i < N) {
        float best = sD[r][0];
        int lab = 0;
        for (int j = 1; j < k; j++)
            if (sD[r][j] < best) {
                best = sD[r][j];
                lab = j;
            }
        if (labels[i] != lab) atomicAdd(changed, 1ull);
        labels[i] = lab;
    }
}

// M-step sums in sklearn's single-thread order.  _update_chunk_dense (_k_means_lloyd.pyx:
// 210-215) adds every row into its cluster's fp32 row in row order (chunks of 256 rows are
// visited in order; with one OpenMP thread the thread-local buffer is the whole sum), so
// sums[j][d] = (((0 + x_a[d]) + x_b[d]) + ...) over the rows a < b < ... labelled j.  A
// sequential fp32 sum per (cluster, feature) is reproduced exactly by walking each cluster's
// rows in increasing order: a stable counting sort of the rows by label (64-row segments:
// per-segment counts by wave ballots, a per-cluster scan, a ranked scatter), then one wave per
// (64 features, cluster) streams its rows with 16 loads in flight.  (sklearn with T threads
// reduces T partial sums in lock-acquisition order, which is not reproducible; its rows that
// differ from the one-thread result are recorded by the goldens.)
__global__ __launch_bounds__(256) void k_seg_count(const int32_t* __restrict__ labels, int64_t N, int k,
                                                   int64_t nseg, int32_t* __restrict__ cnt) {
    const int lane = threadIdx.x & 63;
    const int64_t s = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (s >= nseg) return;
    const int64_t i = s * 64 + lane;
    const int l = i < N ? labels[i] : -1;
    for (int j = 0; j < k; j++) {
        uint64_t m = __ballot(l == j);
        if (lane == 0) cnt[(int64_t)j * nseg + s] = __popcll(m);
    }
}

// one block, thread j < k: counts -> exclusive offsets (cluster base + running segment sum)
__global__ void k_seg_scan(int32_t* __restrict__ cnt, int k, int64_t nseg, int32_t* __restrict__ csize) {
    __shared__ int64_t tot[64];
    const int j = threadIdx.x;
    int64_t t = 0;
    if (j < k)
        for (int64_t s = 0; s < nseg; s++) t += cnt[(int64_t)j * nseg + s];
    tot[j] = t;
    __syncthreads();
    if (j >= k) return;
    int64_t base = 0;
    for (int q = 0; q < j; q++) base += tot[q];
    csize[j] = (int32_t)t;
    csize[64 + j] = (int32_t)base;
    for (int64_t s = 0; s < nseg; s++) {
        int32_t c = cnt[(int64_t)j * nseg + s];
        cnt[(int64_t)j * nseg + s] = (int32_t)base;
        base += c;
    }
}

__global__ __launch_bounds__(256) void k_seg_scatter(const int32_t* __restrict__ labels, int64_t N, int k,
                                                     int64_t nseg, const int32_t* __restrict__ off,
                                                     int32_t* __restrict__ order) {
    const int lane = threadIdx.x & 63;
    const int64_t s = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    if (s >= nseg) return;
    const int64_t i = s * 64 + lane;
    const int l = i < N ? labels[i] : -1;
    const uint64_t below = (1ull << lane) - 1;
    for (int j = 0; j < k; j++) {
        uint64_t m = __ballot(l == j);
        if (l == j) order[off[(int64_t)j * nseg + s] + __popcll(m & below)] = (int32_t)i;
    }
}

// grid (cdiv(D, 64), k), one wave per block: sums[j][d] = sequential fp32 sum over the
// cluster's rows (order[csize[64+j] ...]) in row order; weights[j] = row count (exact < 2^24)
__global__ __launch_bounds__(64) void k_msum_seq(const float* __restrict__ X, int D, const int32_t* __restrict__ order,
                                                 const int32_t* __restrict__ csize, float* __restrict__ sums,
                                                 float* __restrict__ w) {
    constexpr int U = 16;
    const int j = blockIdx.y;
    const int d = blockIdx.x * 64 + threadIdx.x;
    const int n = csize[j];
    const int32_t* rows = order + csize[64 + j];
    const bool ok = d < D;
    const float* xcol = X + (ok ? d : 0);
    float acc = 0.f;
    int t = 0;
    for (; t + U <= n; t += U) {
        float v[U];
#pragma unroll
        for (int u = 0; u < U; u++) v[u] = xcol[(int64_t)rows[t + u] * D];
#pragma unroll
        for (int u = 0; u < U; u++) acc += v[u];
    }
    for (; t < n; t++) acc += xcol[(int64_t)rows[t] * D];
    if (ok) sums[(int64_t)j * D + d] = acc;
    if (blockIdx.x == 0 && threadIdx.x == 0) w[j] = (float)n;
}

// _average_centers + _center_shift (_k_means_common.pyx:274-311), one block: each thread
// owns feature columns (the reference's sequential j loop, including its copy of the
// argmax-weight center into still-empty clusters), then one thread per cluster for the shift
__global__ void k_average(float* __restrict__ Cn, const float* __restrict__ w, const float* __restrict__ Co, int k,
                          int D, float* __restrict__ shift) {
    int amax = 0;
    for (int j = 1; j < k; j++)
        if (w[j] > w[amax]) amax = j;
    for (int d = threadIdx.x; d < D; d += blockDim.x) {
        for (int j = 0; j < k; j++) {
            float* c = Cn + (int64_t)j * D;
            if (w[j] > 0.f) {
                float alpha = (float)(1.0 / (double)w[j]);  // `floating alpha = 1.0 / weight` (C double)
                c[d] *= alpha;
            } else {
                c[d] = Cn[(int64_t)amax * D + d];
            }
        }
    }
    __syncthreads();
    for (int j = threadIdx.x; j < k; j += blockDim.x) {
        const float* a = Cn + (int64_t)j * D;
        const float* o = Co + (int64_t)j * D;
        float r = 0.f;
        int n4 = D / 4, rem = D % 4, d = 0;
        for (int q = 0; q < n4; q++, d += 4) {
            float t0 = a[d] - o[d], t1 = a[d + 1] - o[d + 1], t2 = a[d + 2] - o[d + 2], t3 = a[d + 3] - o[d + 3];
            r += ((t0 * t0 + t1 * t1) + t2 * t2) + t3 * t3;
        }
        for (int q = 0; q < rem; q++, d++) r += (a[d] - o[d]) * (a[d] - o[d]);
        shift[j] = sqrtf(r);
    }
}

// ((X - centers[labels])**2).sum(axis=1) for empty-cluster relocation
// (_relocate_empty_clusters_dense, _k_means_common.pyx:185): a float32 numpy row sum, i.e.
// numpy's pairwise summation (loops_utils.h: < 8 sequential; <= 128 eight accumulators
// combined ((r0+r1)+(r2+r3))+((r4+r5)+(r6+r7)) then the tail; else halves at a multiple of 8)
struct SqDiff {
    const float* x;
    const float* c;
    __device__ float operator()(int i) const {
        float t = x[i] - c[i];
        return t * t;
    }
};
template <int L>
__device__ float np_pairwise_sum(const SqDiff& f, int off, int n) {
    if (n < 8) {
        float r = 0.f;
        for (int i = 0; i < n; i++) r += f(off + i);
        return r;
    }
    if (n <= 128 || L == 0) {
        float r[8];
#pragma unroll
        for (int q = 0; q < 8; q++) r[q] = f(off + q);
        int i = 8;
        for (; i < n - (n % 8); i += 8)
#pragma unroll
            for (int q = 0; q < 8; q++) r[q] += f(off + i + q);
        float res = ((r[0] + r[1]) + (r[2] + r[3])) + ((r[4] + r[5]) + (r[6] + r[7]));
        for (; i < n; i++) res += f(off + i);
        return res;
    }
    if constexpr (L > 0) {
        int n2 = n / 2;
        n2 -= n2 % 8;
        return np_pairwise_sum<L - 1>(f, off, n2) + np_pairwise_sum<L - 1>(f, off + n2, n - n2);
    }
    return 0.f;
}

__global__ void k_center_dist(const float* __restrict__ X, int64_t N, int D, const float* __restrict__ C,
                              const int32_t* __restrict__ labels, float* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    SqDiff f{X + i * D, C + (int64_t)labels[i] * D};
    out[i] = np_pairwise_sum<14>(f, 0, D);
}

// ------------------------------------------------------------------ pairwise euclidean (N x N)
__global__ void k_rownorm64(const float* __restrict__ X, int64_t N, int D, double* __restrict__ out) {
    int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= N) return;
    double s = 0.0;
    for (int d = 0; d < D; d++) {
        double x = (double)X[i * D + d];
        s += x * x;
    }
    out[i] = s;
}

// 64x64 output tile per 256-thread block, 4x4 doubles per thread, K staged through LDS
__global__ __launch_bounds__(256) void k_pdist(const float* __restrict__ X, int64_t N, int D,
                                               const double* __restrict__ nrm, float* __restrict__ out) {
    constexpr int T = 64, KB = 16;
    __shared__ double sA[KB][T + 1], sB[KB][T + 1];
    const int tx = threadIdx.x & 15, ty = threadIdx.x >> 4;
    const int64_t i0 = (int64_t)blockIdx.y * T, j0 = (int64_t)blockIdx.x * T;
    double acc[4][4] = {};
    for (int k0 = 0; k0 < D; k0 += KB) {
        for (int e = threadIdx.x; e < T * KB; e += 256) {
            int r = e / KB, kk = e % KB;
            int64_t ia = i0 + r, jb = j0 + r;
            sA[kk][r] = (ia < N && k0 + kk < D) ? (double)X[ia * D + k0 + kk] : 0.0;
            sB[kk][r] = (jb < N && k0 + kk < D) ? (double)X[jb * D + k0 + kk] : 0.0;
        }
        __syncthreads();
#pragma unroll
        for (int kk = 0; kk < KB; kk++) {
            double a[4], b[4];
#pragma unroll
            for (int q = 0; q < 4; q++) {
                a[q] = sA[kk][ty + 16 * q];
                b[q] = sB[kk][tx + 16 * q];
            }
#pragma unroll
            for (int p = 0; p < 4; p++)
#pragma unroll
                for (int q = 0; q < 4; q++) acc[p][q] = fma(a[p], b[q], acc[p][q]);
        }
        __syncthreads();
    }
#pragma unroll
    for (int p = 0; p < 4; p++) {
        int64_t i = i0 + ty + 16 * p;
        if (i >= N) continue;
#pragma unroll
        for (int q = 0; q < 4; q++) {
            int64_t j = j0 + tx + 16 * q;
            if (j >= N) continue;
            double dd = -2.0 * acc[p][q];
            dd += nrm[i];
            dd += nrm[j];
            float f = fmaxf((float)dd, 0.f);
            out[i * N + j] = i == j ? 0.f : sqrtf(f);
        }
    }
}

// ------------------------------------------------------------------ silhouette
// one wave per row i: per-cluster sums of D[i, :] (np.bincount, float64) -> float32, then the
// silhouette_samples arithmetic in numpy's dtypes (float32 arrays divided by int64 counts
// through float64; np.maximum; nan_to_num).
template <int KMAX>
__global__ __launch_bounds__(256) void k_silhouette(const float* __restrict__ Dm, int64_t N,
                                                    const int32_t* __restrict__ labels, int k,
                                                    const int64_t* __restrict__ freq, float* __restrict__ sil) {
    const int lane = threadIdx.x & 63;
    const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t i = wid; i < N; i += nw) {
        double acc[KMAX];
#pragma unroll
        for (int c = 0; c < KMAX; c++) acc[c] = 0.0;
        const float* row = Dm + i * N;
        for (int64_t j = lane; j < N; j += 64) {
            double v = (double)row[j];
            int l = labels[j];
#pragma unroll
            for (int c = 0; c < KMAX; c++)
                if (l == c) acc[c] += v;
        }
        float inter = INFINITY, intra = 0.f;
        int li = labels[i];
#pragma unroll
        for (int c = 0; c < KMAX; c++) {
            if (c < k) {
                float cd = (float)wave_sum_f64(acc[c]);
                if (c == li) {
                    intra = cd;
                } else {
                    float m = (float)((double)cd / (double)freq[c]);
                    inter = fminf(inter, m);
                }
            }
        }
        if (lane == 0) {
            float a = (float)((double)intra / (double)(freq[li] - 1));
            float s = inter - a;
            float mx = (isnan(a) || isnan(inter)) ? NAN : fmaxf(a, inter);
            s = s / mx;
            if (isnan(s)) s = 0.f;
            else if (isinf(s)) s = s > 0 ? 3.402823466e38f : -3.402823466e38f;
            sil[i] = s;
        }
    }
}

// ------------------------------------------------------------------ silhouette sweep (no N x N)
// silhouette_samples for M label sets at once, rows [r0, r1) only (a rank's shard), without
// the N x N matrix: sklearn's pairwise_distances_chunked + _silhouette_reduce
// (_unsupervised.py:203-315) computes, per row i and cluster c, the float64 bincount sum of
// D[i, j] over the members j of c, rounded to float32.  Here one workgroup owns 64 rows and
// walks every column tile of 64: the 64 x 64 distance tile (float64 GEMM + norms, fp32, sqrt,
// zero diagonal: k_pdist's formula) goes to LDS, and the per-(row, cluster) sums of every
// label set advance as S += Dt x H, H[j][q] = [label_m(q)(j) == c(q)] over the C = sum k_m
// cluster columns -- a one-hot GEMM in float64 (exact products, double accumulation).  After
// the last tile the sums are rounded to fp32 and each (row, set) gets silhouette_samples'
// arithmetic (k_silhouette).  Memory: O(N D) -- the sweep runs at any N that fits X.
constexpr int SW_T = 64, SW_KB = 16, SW_CMAX = 160, SW_CB = SW_CMAX / 16, SW_MMAX = 32;

struct SilTables {
    int M, C;
    int qm[SW_CMAX], qc[SW_CMAX];  // cluster column -> (set, cluster)
    int off[SW_MMAX], k[SW_MMAX];  // set -> first column, clusters
};

__global__ __launch_bounds__(256) void k_sil_sweep(const float* __restrict__ X, int64_t N, int D,
                                                   const double* __restrict__ nrm, const uint8_t* __restrict__ lab,
                                                   const SilTables tb, const int64_t* __restrict__ freq,
                                                   int64_t r0, int64_t r1, float* __restrict__ sil) {
    // LDS: GEMM staging + distance tile + one-hot tile; reused for the fp32 sums at the end
    constexpr int STAGE = 2 * SW_KB * (SW_T + 1) * 8 + SW_T * (SW_T + 1) * 4 + SW_T * SW_CMAX;
    static_assert(STAGE >= SW_T * SW_CMAX * 4, "sum buffer overlays the staging");
    __shared__ __attribute__((aligned(16))) unsigned char smem[STAGE];
    double (*sA)[SW_T + 1] = reinterpret_cast<double (*)[SW_T + 1]>(smem);
    double (*sB)[SW_T + 1] = reinterpret_cast<double (*)[SW_T + 1]>(smem + SW_KB * (SW_T + 1) * 8);
    float (*Dt)[SW_T + 1] = reinterpret_cast<float (*)[SW_T + 1]>(smem + 2 * SW_KB * (SW_T + 1) * 8);
    uint8_t (*Hs)[SW_CMAX] = reinterpret_cast<uint8_t (*)[SW_CMAX]>(smem + 2 * SW_KB * (SW_T + 1) * 8 +
                                                                     SW_T * (SW_T + 1) * 4);
    const int tid = threadIdx.x, tx = tid & 15, ty = tid >> 4;
    const int64_t i0 = r0 + (int64_t)blockIdx.x * SW_T;
    const int C = tb.C;
    double S[4][SW_CB];
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
        for (int b = 0; b < SW_CB; b++) S[a][b] = 0.0;
    for (int64_t j0 = 0; j0 < N; j0 += SW_T) {
        double acc[4][4] = {};
        for (int k0 = 0; k0 < D; k0 += SW_KB) {
            for (int e = tid; e < SW_T * SW_KB; e += 256) {
                int r = e / SW_KB, kk = e % SW_KB;
                int64_t ia = i0 + r, jb = j0 + r;
                sA[kk][r] = (ia < r1 && k0 + kk < D) ? (double)X[ia * D + k0 + kk] : 0.0;
                sB[kk][r] = (jb < N && k0 + kk < D) ? (double)X[jb * D + k0 + kk] : 0.0;
            }
            __syncthreads();
#pragma unroll
            for (int kk = 0; kk < SW_KB; kk++) {
                double av[4], bv[4];
#pragma unroll
                for (int q = 0; q < 4; q++) {
                    av[q] = sA[kk][ty + 16 * q];
                    bv[q] = sB[kk][tx + 16 * q];
                }
#pragma unroll
                for (int p = 0; p < 4; p++)
#pragma unroll
                    for (int q = 0; q < 4; q++) acc[p][q] = fma(av[p], bv[q], acc[p][q]);
            }
            __syncthreads();
        }
        // distance tile (k_pdist's epilogue) and the one-hot tile of this column block
#pragma unroll
        for (int p = 0; p < 4; p++) {
            int64_t i = i0 + ty + 16 * p;
#pragma unroll
            for (int q = 0; q < 4; q++) {
                int64_t j = j0 + tx + 16 * q;
                float dv = 0.f;
                if (i < r1 && j < N) {
                    double dd = -2.0 * acc[p][q];
                    dd += nrm[i];
                    dd += nrm[j];
                    float f = fmaxf((float)dd, 0.f);
                    dv = i == j ? 0.f : sqrtf(f);
                }
                Dt[ty + 16 * p][tx + 16 * q] = dv;
            }
        }
        for (int e = tid; e < SW_T * C; e += 256) {
            int jj = e / C, q = e % C;
            int64_t j = j0 + jj;
            Hs[jj][q] = (j < N && lab[(int64_t)tb.qm[q] * N + j] == tb.qc[q]) ? 1 : 0;
        }
        __syncthreads();
        // S[rows ty + 16a][cols tx + 16b] += sum_j Dt[row][j] * H[j][col]
        const int jn = (int)min<int64_t>(SW_T, N - j0);
        for (int jj = 0; jj < jn; jj++) {
            double dv[4];
#pragma unroll
            for (int a = 0; a < 4; a++) dv[a] = (double)Dt[ty + 16 * a][jj];
#pragma unroll
            for (int b = 0; b < SW_CB; b++) {
                int q = tx + 16 * b;
                if (q < C && Hs[jj][q]) {
#pragma unroll
                    for (int a = 0; a < 4; a++) S[a][b] += dv[a];
                }
            }
        }
        __syncthreads();
    }
    // fp32 sums (cluster_distances is a float32 array) -> LDS, then silhouette per (row, set)
    float (*Sf)[SW_CMAX] = reinterpret_cast<float (*)[SW_CMAX]>(smem);
#pragma unroll
    for (int a = 0; a < 4; a++)
#pragma unroll
        for (int b = 0; b < SW_CB; b++) {
            int q = tx + 16 * b;
            if (q < C) Sf[ty + 16 * a][q] = (float)S[a][b];
        }
    __syncthreads();
    for (int e = tid; e < SW_T * tb.M; e += 256) {
        int r = e % SW_T, m = e / SW_T;
        int64_t i = i0 + r;
        if (i >= r1) continue;
        const int li = lab[(int64_t)m * N + i], o = tb.off[m];
        const int64_t* fr = freq + o;
        float inter = INFINITY, intra = 0.f;
        for (int c = 0; c < tb.k[m]; c++) {
            float cd = Sf[r][o + c];
            if (c == li) {
                intra = cd;
            } else {
                float mm = (float)((double)cd / (double)fr[c]);
                inter = fminf(inter, mm);
            }
        }
        float a = (float)((double)intra / (double)(fr[li] - 1));
        float sv = inter - a;
        float mx = (isnan(a) || isnan(inter)) ? NAN : fmaxf(a, inter);
        sv = sv / mx;
        if (isnan(sv)) sv = 0.f;
        else if (isinf(sv)) sv = sv > 0 ? 3.402823466e38f : -3.402823466e38f;
        sil[(int64_t)m * (r1 - r0) + (i - r0)] = sv;
    }
}

// ------------------------------------------------------------------ cluster statistics (CH, DB)
// sums[k][D] (double), sqn[k] = sum |x|^2 (double), cnt[k]: one block per row chunk,
// atomics on double (order-independent up to float64 rounding)
__global__ void k_csum(const float* __restrict__ X, int64_t N, int D, const int32_t* __restrict__ labels,
                       double* __restrict__ sums, double* __restrict__ sqn, unsigned long long* __restrict__ cnt) {
    int64_t i = blockIdx.x;
    if (i >= N) return;
    int l = labels[i];
    double q = 0.0;
    for (int d = threadIdx.x; d < D; d += blockDim.x) {
        double x = (double)X[i * D + d];
        atomicAdd(&sums[(int64_t)l * D + d], x);
        q += x * x;
    }
    __shared__ double red[256];
    red[threadIdx.x] = q;
    __syncthreads();
    for (int s = blockDim.x / 2; s > 0; s >>= 1) {
        if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        atomicAdd(&sqn[l], red[0]);
        atomicAdd(&cnt[l], 1ull);
    }
}

// dsum[k] += |x_i - centroid_{l_i}| (float64), Davies-Bouldin intra distances
__global__ void k_cdist(const float* __restrict__ X, int64_t N, int D, const int32_t* __restrict__ labels,
                        const double* __restrict__ cent, double* __restrict__ dsum) {
    const int lane = threadIdx.x & 63;
    const int64_t wid = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t nw = ((int64_t)gridDim.x * blockDim.x) >> 6;
    for (int64_t i = wid; i < N; i += nw) {
        int l = labels[i];
        double s = 0.0;
        for (int d = lane; d < D; d += 64) {
            double t = (double)X[i * D + d] - cent[(int64_t)l * D + d];
            s += t * t;
        }
        s = wave_sum_f64(s);
        if (lane == 0) atomicAdd(&dsum[l], sqrt(s));
    }
}

struct Group {
    int device = 0;
    hipStream_t st = 0;
    Arena ar;
};

static int waves_grid(int64_t n) { return (int)std::min<int64_t>(cdiv(n, 4), 256 * 16); }

}  // namespace vtf

using namespace vtf;

struct vtf_group_s {
    Group g;
};

extern "C" {

int vtf_group_create(int device, vtf_group_t* out) {
    return guarded([&] {
        VTF_CHECK(out, VTF_E_ARG, "null argument");
        DeviceGuard dg(device);
        auto* h = new vtf_group_s();
        h->g.device = device;
        *out = h;
    });
}

int vtf_group_destroy(vtf_group_t h) {
    return guarded_on(h ? h->g.device : -1, [&] { delete h; });
}

int vtf_group_set_stream(vtf_group_t h, void* stream) {
    return guarded_on(h ? h->g.device : -1, [&] {
        VTF_CHECK(h, VTF_E_ARG, "null handle");
        h->g.st = (hipStream_t)stream;
    });
}

int vtf_colstats(vtf_group_t h, const float* d_X, int64_t N, int64_t D, float* d_Xc, float* d_mean, float* d_var) {
    return guarded_on(h ? h->g.device : -1, [&] {
        VTF_CHECK(h && d_X && d_mean && d_var && N > 0 && D > 0 && D < (1 << 20), VTF_E_ARG, "bad argument");
        k_colstats<<<cdiv(D, 64), 64, 0, h->g.st>>>(d_X, N, (int)D, d_Xc, d_mean, d_var);
        VTF_HIP(hipGetLastError());
    });
}

int vtf_sqdist_rows(vtf_group_t h, const float* d_X, int64_t N, int64_t D, const int64_t* rows, int T, float* d_out) {
    return guarded_on(h ? h->g.device : -1, [&] {
        VTF_CHECK(h && d_X && rows && d_out && N > 0 && D > 0 && T > 0 && T <= 16, VTF_E_ARG, "bad argument");
        VTF_CHECK((size_t)T * D * 4 <= 64 * 1024, VTF_E_LIMIT, "sqdist_rows: T*D too large");
        for (int t = 0; t < T; t++) VTF_CHECK(rows[t] >= 0 && rows[t] < N, VTF_E_ARG, "row index out of range");
        int64_t* dr = h->g.ar.get<int64_t>(0, T);
        VTF_HIP(hipMemcpyAsync(dr, rows, T * 8, hipMemcpyHostToDevice, h->g.st));
        size_t sh = (size_t)T * D * 4;
        if (T <= 4)
            k_sqdist_rows<4><<<waves_grid(N), 256, sh, h->g.st>>>(d_X, N, (int)D, dr, T, d_out);
        else
            k_sqdist_rows<16><<<waves_grid(N), 256, sh, h->g.st>>>(d_X, N, (int)D, dr, T, d_out);
        VTF_HIP(hipGetLastError());
        VTF_HIP(hipStreamSynchronize(h->g.st));
    });
}

// E-step (+ M-step sums when d_sums != NULL).  d_labels in/out; *out_changed = labels changed.
int vtf_kmeans_step(vtf_group_t h, const float* d_X, int64_t N, int64_t D, const float* d_centers, int k,
                    int32_t* d_labels, float* d_sums, float* d_weights, int64_t* out_changed) {
    return guarded_on(h ? h->g.device : -1, [&] {
        VTF_CHECK(h && d_X && d_centers && d_labels && N > 0 && D > 0 && k > 0, VTF_E_ARG, "bad argument");
        VTF_CHECK(k <= 64, VTF_E_LIMIT, "kmeans: at most 64 clusters (the E-step keeps every center's distance in LDS)");
        Group& G = h->g;
        float* csq = G.ar.get<float>(1, k);
        unsigned long long* chg = G.ar.get<unsigned long long>(2, 1);
        VTF_HIP(hipMemsetAsync(chg, 0, 8, G.st));
        k_csq<<<cdiv(k, 64), 64, 0, G.st>>>(d_centers, k, (int)D, csq);
        k_estep<<<(unsigned)cdiv(N, ES_R), 256, 0, G.st>>>(d_X, N, (int)D, d_centers, csq, k, d_labels, chg);
        if (d_sums) {
            VTF_CHECK(d_weights, VTF_E_ARG, "null weights");
            VTF_CHECK(k <= 64, VTF_E_LIMIT, "kmeans: k > 64");
            VTF_CHECK(N < (1 << 24), VTF_E_LIMIT, "kmeans: N >= 2^24 (fp32 row counts)");
            const int64_t nseg = cdiv(N, 64);
            int32_t* cnt = G.ar.get<int32_t>(3, (size_t)nseg * k);
            int32_t* order = G.ar.get<int32_t>(4, (size_t)N);
            int32_t* csize = G.ar.get<int32_t>(6, 128);
            const unsigned sg = (unsigned)cdiv(nseg, 4);
            k_seg_count<<<sg, 256, 0, G.st>>>(d_labels, N, k, nseg, cnt);
            k_seg_scan<<<1, 64, 0, G.st>>>(cnt, k, nseg, csize);
            k_seg_scatter<<<sg, 256, 0, G.st>>>(d_labels, N, k, nseg, cnt, order);
            k_msum_seq<<<dim3(cdiv(D, 64), k), 64, 0, G.st>>>(d_X, (int)D, order, csize, d_sums, d_weights);
        }
        unsigned long long c = 0;
        VTF_HIP(hipMemcpyAsync(&c, chg, 8, hipMemcpyDeviceToHost, G.st));
        VTF_HIP(hipStreamSynchronize(G.st));
        if (out_changed) *out_changed = (int64_t)c;
    });
}

int vtf_kmeans_average(vtf_group_t h, float* d_sums, const float* d_weights, const float* d_centers_old, int k,
                       int64_t D, float* d_shift) {
    return guarded_on(h ? h->g.device : -1, [&] {
        VTF_CHECK(h && d_sums && d_weights && d_centers_old && d_shift && k > 0 && D > 0, VTF_E_ARG, "bad argument");
        k_average<<<1, 256, 0, h->g.st>>>(d_sums, d_weights, d_centers_old, k, (int)D, d_shift);
        VTF_HIP(hipGetLastError());
    });
}

int vtf_center_dist(vtf_group_t h, const float* d_X, int64_t N, int64_t D, const float* d_centers,
                    const int32_t* d_labels, float* d_out) {
    return guarded_on(h ? h->g.device : -1, [&] {
        VTF_CHECK(h && d_X && d_centers && d_labels && d_out && N > 0 && D > 0, VTF_E_ARG, "bad argument");
        k_center_dist<<<cdiv(N, 256), 256, 0, h->g.st>>>(d_X, N, (int)D, d_centers, d_labels, d_out);
        VTF_HIP(hipGetLastError());
    });
}

int vtf_pairwise_euclidean(vtf_group_t h, const float* d_X, int64_t N, int64_t D, float* d_out) {
    return guarded_on(h ? h->g.device : -1, [&] {
        VTF_CHECK(h && d_X && d_out && N > 0 && D > 0, VTF_E_ARG, "bad argument");
        VTF_CHECK(N <= (1 << 20), VTF_E_LIMIT, "pairwise: N too large");
        double* nrm = h->g.ar.get<double>(5, N);
        k_rownorm64<<<cdiv(N, 256), 256, 0, h->g.st>>>(d_X, N, (int)D, nrm);
        dim3 grid(cdiv(N, 64), cdiv(N, 64));
        k_pdist<<<grid, 256, 0, h->g.st>>>(d_X, N, (int)D, nrm, d_out);
        VTF_HIP(hipGetLastError());
    });
}

int vtf_silhouette_samples(vtf_group_t h, const float* d_D, int64_t N, const int32_t* d_labels, int k,
                           const int64_t* d_freq, float* d_sil) {
    return guarded_on(h ? h->g.device : -1, [&] {
        VTF_CHECK(h && d_D && d_labels && d_freq && d_sil && N > 1 && k >= 2, VTF_E_ARG, "bad argument");
        VTF_CHECK(k <= 64, VTF_E_LIMIT, "silhouette: more than 64 labels");
        hipStream_t st = h->g.st;
        int grid = waves_grid(N);
        if (k <= 8)
            k_silhouette<8><<<grid, 256, 0, st>>>(d_D, N, d_labels, k, d_freq, d_sil);
        else if (k <= 16)
            k_silhouette<16><<<grid, 256, 0, st>>>(d_D, N, d_labels, k, d_freq, d_sil);
        else if (k <= 32)
            k_silhouette<32><<<grid, 256, 0, st>>>(d_D, N, d_labels, k, d_freq, d_sil);
        else
            k_silhouette<64><<<grid, 256, 0, st>>>(d_D, N, d_labels, k, d_freq, d_sil);
        VTF_HIP(hipGetLastError());
    });
}

int vtf_silhouette_sweep(vtf_group_t h, const float* d_X, int64_t N, int64_t D, int64_t row_begin, int64_t row_end,
                         const uint8_t* d_labels, int M, const int32_t* ks, const int64_t* freq, float* d_sil) {
    return guarded_on(h ? h->g.device : -1, [&] {
        VTF_CHECK(h && d_X && d_labels && ks && freq && d_sil && N > 1 && D > 0 && M > 0, VTF_E_ARG, "bad argument");
        VTF_CHECK(0 <= row_begin && row_begin <= row_end && row_end <= N, VTF_E_ARG, "bad row range");
        VTF_CHECK(M <= SW_MMAX, VTF_E_LIMIT, "silhouette_sweep: more than 32 label sets");
        SilTables tb{};
        tb.M = M;
        int C = 0;
        for (int m = 0; m < M; m++) {
            VTF_CHECK(ks[m] >= 2 && ks[m] <= 255, VTF_E_ARG, "label set with fewer than 2 or more than 255 labels");
            tb.off[m] = C;
            tb.k[m] = ks[m];
            VTF_CHECK(C + ks[m] <= SW_CMAX, VTF_E_LIMIT, "silhouette_sweep: more than 160 clusters in one pass");
            for (int c = 0; c < ks[m]; c++, C++) {
                tb.qm[C] = m;
                tb.qc[C] = c;
            }
        }
        tb.C = C;
        if (row_end == row_begin) return;
        Group& G = h->g;
        double* nrm = G.ar.get<double>(5, N);
        int64_t* dfreq = G.ar.get<int64_t>(7, C);
        VTF_HIP(hipMemcpyAsync(dfreq, freq, (size_t)C * 8, hipMemcpyHostToDevice, G.st));
        k_rownorm64<<<cdiv(N, 256), 256, 0, G.st>>>(d_X, N, (int)D, nrm);
        k_sil_sweep<<<cdiv(row_end - row_begin, SW_T), 256, 0, G.st>>>(d_X, N, (int)D, nrm, d_labels, tb, dfreq,
                                                                       row_begin, row_end, d_sil);
        VTF_HIP(hipGetLastError());
        VTF_HIP(hipStreamSynchronize(G.st));  // the host freq buffer may go away after return
    });
}

int vtf_cluster_sums(vtf_group_t h, const float* d_X, int64_t N, int64_t D, const int32_t* d_labels, int k,
                     double* d_sums, double* d_sqnorm, int64_t* d_counts) {
    return guarded_on(h ? h->g.device : -1, [&] {
        VTF_CHECK(h && d_X && d_labels && d_sums && d_sqnorm && d_counts && N > 0 && D > 0 && k > 0, VTF_E_ARG,
                  "bad argument");
        hipStream_t st = h->g.st;
        VTF_HIP(hipMemsetAsync(d_sums, 0, (size_t)k * D * 8, st));
        VTF_HIP(hipMemsetAsync(d_sqnorm, 0, (size_t)k * 8, st));
        VTF_HIP(hipMemsetAsync(d_counts, 0, (size_t)k * 8, st));
        k_csum<<<(unsigned)N, 256, 0, st>>>(d_X, N, (int)D, d_labels, d_sums, d_sqnorm,
                                           (unsigned long long*)d_counts);
        VTF_HIP(hipGetLastError());
    });
}

int vtf_cluster_dist(vtf_group_t h, const float* d_X, int64_t N, int64_t D, const int32_t* d_labels, int k,
                     const double* d_centroids, double* d_dsum) {
    return guarded_on(h ? h->g.device : -1, [&] {
        VTF_CHECK(h && d_X && d_labels && d_centroids && d_dsum && N > 0 && D > 0 && k > 0, VTF_E_ARG,
                  "bad argument");
        VTF_HIP(hipMemsetAsync(d_dsum, 0, (size_t)k * 8, h->g.st));
        k_cdist<<<waves_grid(N), 256, 0, h->g.st>>>(d_X, N, (int)D, d_labels, d_centroids, d_dsum);
        VTF_HIP(hipGetLastError());
    });
}

}  // extern "C"

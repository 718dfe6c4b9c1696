// Device-wide sort and scan used by the detectors' candidate lists (MTCNN stage-1 order, the IoM
// score order, NMS calls above the segment sort's bound, the R-CNN RPN top-k order) and by every
// flag compaction (MTCNN stage gates, YOLO decode, RPN / RoI filters): hand-written for gfx950 in
// place of rocPRIM's radix sort / merge sort / look-back scan.
//
//   sort_u64_pairs / merge_pairs_u64: (key, value) pairs ascending by (key, value).  Every caller
//     passes values that increase with the input position among equal keys (element indices,
//     positions inside a level), so this IS the stable sort by key that the reference's torch
//     sorts / nonzero orders need.  2048-pair tiles are sorted by one 256-thread workgroup each
//     (bitonic network on the pair order, padding = +inf: in registers, across lanes by shuffles,
//     across waves through LDS), then ceil(log2(tiles)) merge
//     passes: each thread finds its 8-output window of a run pair by a merge-path binary search
//     and merges it sequentially (no atomics, no look-back: nothing waits on another workgroup,
//     so the passes do not stall behind other lanes' persistent kernels).
//   inclusive_scan_i32: up to 8192 elements one workgroup; above, per-tile sums -> one
//     workgroup scans the sums -> every tile scans itself from its offset (3 launches).
#include <climits>

#include "common.hpp"
#include "nms.hpp"

namespace vtf {

// tile sort: 256 threads x 8 pairs = 2048-pair tiles (24 KB of LDS for the cross-wave stages).
// Small on purpose: a 1024-thread, 48-KB workgroup found no room next to a running k_pnet (its
// four workgroups fill a CU's LDS and registers) and waited ~0.75 ms per sort under four
// pipeline lanes; 256 threads with <= 38 KB fit beside three of them.
constexpr int PS_T = 256, PS_E = 8, PS_TILE = PS_T * PS_E;
constexpr int PM_E = 8, PM_T = 256;  // merge pass: outputs per thread, threads per block

__device__ inline bool pair_lt(uint64_t ka, int32_t va, uint64_t kb, int32_t vb) {
    return ka < kb || (ka == kb && va < vb);
}

// bitonic network over the tile: thread t holds pairs 8 t .. 8 t + 7 in registers.  Partner
// distance j < 8: inside the thread; 8 <= j < 512: another lane of the same wave (lane ^ j / 8,
// shuffles); j >= 512: another wave (the pairs through LDS, one barrier per distance)
__global__ __launch_bounds__(PS_T) void k_tile_sort(const uint64_t* __restrict__ kin, const int32_t* __restrict__ vin,
                                                    int64_t n, uint64_t* __restrict__ kout, int32_t* __restrict__ vout) {
    __shared__ uint64_t sk[PS_TILE];
    __shared__ int32_t sv[PS_TILE];
    const int tid = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * PS_TILE;
    const int m = (int)min((int64_t)PS_TILE, n - base);
    uint64_t k[PS_E];
    int32_t v[PS_E];
#pragma unroll
    for (int r = 0; r < PS_E; r++) {
        const int i = PS_E * tid + r;
        const bool in = i < m;
        k[r] = in ? kin[base + i] : ~0ull;  // padding sorts last (values: INT_MAX > any index)
        v[r] = in ? vin[base + i] : INT_MAX;
    }
    auto cas = [](uint64_t& ka, int32_t& va, uint64_t& kb, int32_t& vb, bool asc) {
        // (ka, va) <- the smaller of the two when asc, the larger otherwise
        const bool sw = asc ? pair_lt(kb, vb, ka, va) : pair_lt(ka, va, kb, vb);
        if (sw) {
            const uint64_t tk = ka;
            const int32_t tv = va;
            ka = kb, va = vb, kb = tk, vb = tv;
        }
    };
    for (int kk = 2; kk <= PS_TILE; kk <<= 1) {
        int j = kk >> 1;
        if (j >= 64 * PS_E) {
#pragma unroll
            for (int r = 0; r < PS_E; r++) {
                sk[PS_E * tid + r] = k[r];
                sv[PS_E * tid + r] = v[r];
            }
            __syncthreads();
            for (; j >= 64 * PS_E; j >>= 1) {
#pragma unroll
                for (int u = 0; u < PS_TILE / 2 / PS_T; u++) {
                    const int q = tid + PS_T * u;
                    const int i = ((q & ~(j - 1)) << 1) | (q & (j - 1)), p = i | j;
                    uint64_t ka = sk[i], kb = sk[p];
                    int32_t va = sv[i], vb = sv[p];
                    cas(ka, va, kb, vb, (i & kk) == 0);
                    sk[i] = ka, sk[p] = kb;
                    sv[i] = va, sv[p] = vb;
                }
                __syncthreads();
            }
#pragma unroll
            for (int r = 0; r < PS_E; r++) {
                k[r] = sk[PS_E * tid + r];
                v[r] = sv[PS_E * tid + r];
            }
            __syncthreads();  // (the next distance's stores overwrite these slots)
        }
        for (; j >= PS_E; j >>= 1) {
            const int lm = j / PS_E;  // partner lane: lane ^ lm
            const bool lower = (tid & lm) == 0;
#pragma unroll
            for (int r = 0; r < PS_E; r++) {
                const int i = PS_E * tid + r;
                const uint32_t lo = __shfl_xor((uint32_t)k[r], lm), hi = __shfl_xor((uint32_t)(k[r] >> 32), lm);
                const int32_t pv = __shfl_xor(v[r], lm);
                const uint64_t pk = ((uint64_t)hi << 32) | lo;
                const bool asc = (i & kk) == 0;
                // the lower index keeps the smaller pair in an ascending run, the larger otherwise
                const bool take_min = lower == asc;
                const bool p_less = pair_lt(pk, pv, k[r], v[r]);
                if (take_min ? p_less : !p_less) {
                    k[r] = pk;
                    v[r] = pv;
                }
            }
        }
        for (; j > 0; j >>= 1) {
#pragma unroll
            for (int r = 0; r < PS_E; r++)
                if ((r & j) == 0) cas(k[r], v[r], k[r | j], v[r | j], ((PS_E * tid + r) & kk) == 0);
        }
    }
#pragma unroll
    for (int r = 0; r < PS_E; r++) {
        const int i = PS_E * tid + r;
        if (i < m) {
            kout[base + i] = k[r];
            vout[base + i] = v[r];
        }
    }
}

// sorted runs of width w -> runs of 2 w: output positions [PM_E t, PM_E (t + 1)) of thread t
__global__ __launch_bounds__(PM_T) void k_merge_pass(const uint64_t* __restrict__ ki, const int32_t* __restrict__ vi,
                                                     int64_t n, int64_t w, uint64_t* __restrict__ ko,
                                                     int32_t* __restrict__ vo) {
    const int64_t o0 = ((int64_t)blockIdx.x * PM_T + threadIdx.x) * PM_E;
    if (o0 >= n) return;
    const int64_t a0 = o0 / (2 * w) * (2 * w), a1 = min(a0 + w, n), b1 = min(a0 + 2 * w, n);
    const int64_t na = a1 - a0, nb = b1 - a1, d = o0 - a0;
    // i = elements of run A among the first d outputs (A first on equal pairs: stable)
    int64_t lo = max((int64_t)0, d - nb), hi = min(d, na);
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        const int64_t bj = a1 + d - 1 - mid;
        if (!pair_lt(ki[bj], vi[bj], ki[a0 + mid], vi[a0 + mid])) lo = mid + 1; else hi = mid;
    }
    int64_t ia = a0 + lo, ib = a1 + (d - lo);
    const int64_t oe = min(o0 + PM_E, b1);
    for (int64_t o = o0; o < oe; o++) {
        bool takeA = ib >= b1;
        if (!takeA && ia < a1) takeA = !pair_lt(ki[ib], vi[ib], ki[ia], vi[ia]);
        if (takeA) {
            ko[o] = ki[ia];
            vo[o] = vi[ia];
            ia++;
        } else {
            ko[o] = ki[ib];
            vo[o] = vi[ib];
            ib++;
        }
    }
}

void sort_u64_pairs(Arena& ar, int slot, const uint64_t* kin, uint64_t* kout, const int32_t* vin, int32_t* vout,
                    int64_t n, int end_bit, hipStream_t st) {
    (void)end_bit;  // (the comparison covers the whole key)
    if (n <= 0) return;
    VTF_CHECK(n < ((int64_t)1 << 31), VTF_E_LIMIT, "sort: too many pairs");
    const int64_t tiles = (n + PS_TILE - 1) / PS_TILE;
    int passes = 0;
    while (((int64_t)PS_TILE << passes) < n) passes++;
    // the tile sort writes where the last merge pass must not read: kout after an even count
    uint64_t* kt = passes ? (uint64_t*)ar.get(slot, (size_t)n * 12 + 16) : nullptr;
    int32_t* vt = passes ? (int32_t*)(kt + n) : nullptr;
    uint64_t* kb[2] = {kout, kt};
    int32_t* vb[2] = {vout, vt};
    int cur = passes & 1;
    k_tile_sort<<<(unsigned)tiles, PS_T, 0, st>>>(kin, vin, n, kb[cur], vb[cur]);
    for (int p = 0; p < passes; p++) {
        const int64_t w = (int64_t)PS_TILE << p;
        k_merge_pass<<<(unsigned)cdiv(cdiv(n, PM_E), PM_T), PM_T, 0, st>>>(kb[cur], vb[cur], n, w, kb[cur ^ 1], vb[cur ^ 1]);
        cur ^= 1;
    }
    VTF_HIP(hipGetLastError());
}

void merge_pairs_u64(Arena& ar, int slot, const uint64_t* kin, uint64_t* kout, const int32_t* vin, int32_t* vout,
                     int64_t n, hipStream_t st) {
    sort_u64_pairs(ar, slot, kin, kout, vin, vout, n, 64, st);
}

// ------------------------------------------------------------------------------------- scan
constexpr int SC_T = 1024, SC_E = 8, SC_TILE = SC_T * SC_E;

// exclusive scan of one value per thread over the workgroup (1024 threads); returns the total
__device__ inline int block_excl(int v, int* wsum, int& total) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    int x = v;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) wsum[wave] = x;
    __syncthreads();
    if (tid < 64) {
        const int s = tid < SC_T / 64 ? wsum[tid] : 0;
        int t = s;
#pragma unroll
        for (int o = 1; o < 16; o <<= 1) {
            const int y = __shfl_up(t, o);
            if (lane >= o) t += y;
        }
        if (tid < SC_T / 64) wsum[tid] = t - s;
        if (tid == SC_T / 64 - 1) wsum[SC_T / 64] = t;
    }
    __syncthreads();
    total = wsum[SC_T / 64];
    return wsum[wave] + x - v;
}

// inclusive scan of tile blockIdx.x from `off` (tile offsets, or none): elements are staged in
// LDS with coalesced loads, each thread scans SC_E consecutive ones
__global__ __launch_bounds__(SC_T) void k_scan_tile(const int32_t* __restrict__ in, int32_t* __restrict__ out, int64_t n,
                                                    const int32_t* __restrict__ off) {
    __shared__ int32_t s[SC_TILE];
    __shared__ int wsum[SC_T / 64 + 1];
    const int tid = threadIdx.x;
    const int64_t base = (int64_t)blockIdx.x * SC_TILE;
    const int m = (int)min((int64_t)SC_TILE, n - base);
    for (int i = tid; i < SC_TILE; i += SC_T) s[i] = i < m ? in[base + i] : 0;
    __syncthreads();
    int v[SC_E], t = 0;
#pragma unroll
    for (int e = 0; e < SC_E; e++) v[e] = (t += s[tid * SC_E + e]);
    int total;
    const int ex = block_excl(t, wsum, total) + (off ? off[blockIdx.x] : 0);
#pragma unroll
    for (int e = 0; e < SC_E; e++) s[tid * SC_E + e] = v[e] + ex;
    __syncthreads();
    for (int i = tid; i < m; i += SC_T) out[base + i] = s[i];
}

__global__ __launch_bounds__(SC_T) void k_tile_sums(const int32_t* __restrict__ in, int64_t n, int32_t* __restrict__ sums) {
    __shared__ int wsum[SC_T / 64 + 1];
    const int64_t base = (int64_t)blockIdx.x * SC_TILE;
    int t = 0;
    for (int i = threadIdx.x; i < SC_TILE; i += SC_T)
        if (base + i < n) t += in[base + i];
    int total;
    block_excl(t, wsum, total);
    if (threadIdx.x == 0) sums[blockIdx.x] = total;
}

// exclusive scan of the tile sums in place (one workgroup, chunks of SC_T with a carry)
__global__ __launch_bounds__(SC_T) void k_scan_sums(int32_t* __restrict__ sums, int64_t nt) {
    __shared__ int wsum[SC_T / 64 + 1];
    int carry = 0;
    for (int64_t c0 = 0; c0 < nt; c0 += SC_T) {
        const int64_t i = c0 + threadIdx.x;
        const int v = i < nt ? sums[i] : 0;
        int total;
        const int ex = block_excl(v, wsum, total);
        if (i < nt) sums[i] = carry + ex;
        carry += total;
        __syncthreads();  // wsum is reused by the next chunk
    }
}

void inclusive_scan_i32(Arena& ar, int slot, const int32_t* in, int32_t* out, int64_t n, hipStream_t st) {
    if (n <= 0) return;
    const int64_t nt = (n + SC_TILE - 1) / SC_TILE;
    VTF_CHECK(nt < ((int64_t)1 << 31), VTF_E_LIMIT, "scan: too many elements");
    if (nt == 1) {
        k_scan_tile<<<1, SC_T, 0, st>>>(in, out, n, nullptr);
    } else {
        int32_t* sums = ar.get<int32_t>(slot, nt);
        k_tile_sums<<<(unsigned)nt, SC_T, 0, st>>>(in, n, sums);
        k_scan_sums<<<1, SC_T, 0, st>>>(sums, nt);
        k_scan_tile<<<(unsigned)nt, SC_T, 0, st>>>(in, out, n, sums);
    }
    VTF_HIP(hipGetLastError());
}

}  // namespace vtf

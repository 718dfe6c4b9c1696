// Implicit-GEMM convolution with LDS-DMA operand staging (gfx950): k_conv's successor for the
// bf16 (perf) mode and for the fp32-grade split-fp16 mode on pre-split operands.
//
// Same GEMM view and epilogue as k_conv (conv.hip): M = N*OH*OW output pixels, N = Cout,
// K = KH*KW*Cin with k = (kh, kw, ci); A is gathered from the NHWC input on the fly, B is the
// weight matrix [Cout][K].  What changes is the staging: every operand piece is 16 bytes =
// 8 consecutive channels of one input pixel (Cin % 8 == 0), and goes HBM -> LDS by one lane of
// a global_load_lds_dwordx4 -- no staging registers, no VALU conversion, no ds_write.  A piece
// that lies in the zero padding, past K or past M is read from a 16-byte zero page instead
// (the per-lane source address makes the im2col gather free).
//
//   MODE 0 (bf16): a k-step is 64 deep; LDS row = 8 chunks of 8 bf16; per fragment pair two
//                  v_mfma_f32_16x16x32_bf16 (k 0..31, 32..63: k_conv's bf16 order, same bits)
//   MODE 1 (split): operands in the split-pair layout (gemm_x3.hpp: x = x0 + x1 2^-11, fp16
//                  pairs), a k-step is 32 deep; LDS row = 4 chunks x 2 planes; per fragment pair
//                  three v_mfma_f32_16x16x32_f16 (x0 w0 | x0 w1 + x1 w0: k_conv's split chains,
//                  same bits when the K loop is not split)
//
// LDS image (both modes): rows of 128 B, 16-B slot s of row r holds source slot s ^ ((r >> 1) & 7),
// written lane-linearly by the DMA (1 KB = 8 rows per wave-instruction; the swizzle is applied
// to the source address), read conflict-free by ds_read_b128 fragment loads.  Two stages (the
// DMA of step k+1 in flight during step k), one barrier per step, two workgroups per CU.
// Grids past a whole round of workgroup slots split their last tiles along K, grids below one
// round split every tile (bf16, or callers that accept a slice-order reduction: split_fp32);
// k_conv_dma_tail sums the slices in order and runs the epilogue.
#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <type_traits>
#include <vector>

#include "common.hpp"
#include "conv.hpp"
#include "conv_dev.hpp"

namespace vtf {

namespace {

typedef __attribute__((ext_vector_type(8))) _Float16 h8;
typedef __attribute__((ext_vector_type(4))) float f4;

template <int MODE, int BM, int BN, int WGM, int OCC = 2, int NSTG = 2>
struct DCfg {
    static constexpr int NS = NSTG;  // LDS stages: NS - 1 k-steps in flight ahead of the MFMAs
    static constexpr int WGN = 4 / WGM, WM = BM / WGM, WN = BN / WGN, FM = WM / 16, FN = WN / 16;
    static constexpr int RB = 128, A_ST = BM * RB, ST = (BM + BN) * RB, LDE = BN + 4;
    static constexpr int SM = NS * ST > BM * LDE * 4 ? NS * ST : BM * LDE * 4;
    static constexpr int PA = BM / 32, PB = BN / 32;  // 1-KB DMA pieces per wave and stage
    static constexpr int CPS = MODE == 1 ? 4 : 8;     // 8-element chunks per k-step
    static constexpr int EB = MODE == 1 ? 4 : 2;      // global bytes per element
    static constexpr int CB = 8 * EB;                 // global bytes per chunk
    static constexpr int KS = 8 * CPS;                // k per step
    static_assert(FM >= 1 && FN >= 1 && BM % 32 == 0 && BN % 32 == 0 && SM * OCC <= 160 * 1024, "tile config");
};

// the tile of work item bid: whole tiles dealt XCD-aware (each XCD owns a contiguous run of
// tile ids; ids walk groups of group_m M-tiles x all N-tiles), then the K slices of the tail tiles
__device__ inline void work_item(const ConvParams& p, int bid, int& t, int& slice, bool& tail) {
    tail = bid >= p.dp_tiles;
    slice = 0;
    if (!tail) {
        const int xcd = bid & 7, loc = bid >> 3, per = p.dp_tiles >> 3, rem = p.dp_tiles & 7;
        t = xcd < rem ? xcd * (per + 1) + loc : rem * (per + 1) + (xcd - rem) * per + loc;
    } else {
        t = p.dp_tiles + (bid - p.dp_tiles) / p.tail_split;
        slice = (bid - p.dp_tiles) % p.tail_split;
    }
}
__device__ inline void tile_of(const ConvParams& p, int t, int& tile_m, int& tile_n) {
    const int gm = p.group_m > 0 ? p.group_m : p.gx;
    const int span = gm * p.gy, first = (t / span) * gm, gsz = min(p.gx - first, gm);
    tile_m = first + (t % span) % gsz;
    tile_n = (t % span) / gsz;
}

// epilogue of `rows` rows of the LDS tile image E [rows][BN + 4] starting at output row m0
template <typename T, int BN>
__device__ inline void dma_epilogue(const ConvParams& p, const float* E, int rows, int64_t m0, int n0) {
    constexpr int LDE = BN + 4, G = BN / 8;
    static_assert(256 % G == 0, "epilogue groups");
    const int tid = threadIdx.x, g = tid % G, c0 = n0 + 8 * g;
    bool bad = false;
    if (c0 < p.Cout) {
        float b8[8], al8[8], be8[8], pr8[8];
#pragma unroll
        for (int e = 0; e < 8; e++) {
            b8[e] = p.bias ? p.bias[c0 + e] : 0.f;
            al8[e] = p.alpha ? p.alpha[c0 + e] : 1.f;
            be8[e] = p.alpha ? p.beta[c0 + e] : 0.f;
            pr8[e] = p.prelu ? p.prelu[c0 + e] : 0.f;
        }
        for (int r = tid / G; r < rows; r += 256 / G) {
            const int64_t m = m0 + r;
            if (m >= p.M) break;
            const f4 lo = *(const f4*)(E + r * LDE + 8 * g), hi = *(const f4*)(E + r * LDE + 8 * g + 4);
            float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            conv_epilogue8<T>(p, m, c0, v, b8, al8, be8, pr8, &bad);
        }
    }
    if (p.out_sp && p.ovf && __ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(p.ovf, 1);
}

// the same epilogue over `cols` columns [c_lo, c_lo + cols) of the LDS tile image E [rows][BN + 4]
template <typename T, int BN, int COLS>
__device__ inline void dma_epilogue_cols(const ConvParams& p, const float* E, int rows, int64_t m0, int n0, int c_lo) {
    constexpr int LDE = BN + 4, G = COLS / 8;
    static_assert(256 % G == 0, "epilogue groups");
    const int tid = threadIdx.x, g = tid % G, c0 = n0 + c_lo + 8 * g;
    bool bad = false;
    if (c0 < p.Cout) {
        float b8[8], al8[8], be8[8], pr8[8];
#pragma unroll
        for (int e = 0; e < 8; e++) {
            b8[e] = p.bias ? p.bias[c0 + e] : 0.f;
            al8[e] = p.alpha ? p.alpha[c0 + e] : 1.f;
            be8[e] = p.alpha ? p.beta[c0 + e] : 0.f;
            pr8[e] = p.prelu ? p.prelu[c0 + e] : 0.f;
        }
        for (int r = tid / G; r < rows; r += 256 / G) {
            const int64_t m = m0 + r;
            if (m >= p.M) break;
            const f4 lo = *(const f4*)(E + r * LDE + c_lo + 8 * g), hi = *(const f4*)(E + r * LDE + c_lo + 8 * g + 4);
            float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
            conv_epilogue8<T>(p, m, c0, v, b8, al8, be8, pr8, &bad);
        }
    }
    if (p.out_sp && p.ovf && __ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(p.ovf, 1);
}

// s_waitcnt vmcnt(N) then the workgroup barrier (LDS reads stay after it)
template <int N>
__device__ inline void wait_vm_barrier() {
    asm volatile("s_waitcnt vmcnt(%0)\n\ts_barrier" ::"n"(N) : "memory");
}

template <int MODE, int BM, int BN, int WGM, int OCC, int NSTG>
__global__ __launch_bounds__(256, OCC) void k_conv_dma(ConvParams p) {
    using C = DCfg<MODE, BM, BN, WGM, OCC, NSTG>;
    using T = typename std::conditional<MODE == 0, __bf16, float>::type;
    constexpr int PA = C::PA, PB = C::PB, FM = C::FM, FN = C::FN, RB = C::RB;
    __shared__ __attribute__((aligned(16))) char smem[C::SM];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / C::WGN, wn = wave % C::WGN;
    int t, slice, tile_m, tile_n;
    bool tail;
    work_item(p, blockIdx.x, t, slice, tail);
    tile_of(p, t, tile_m, tile_n);
    const int64_t m0 = (int64_t)tile_m * BM;
    const int n0 = tile_n * BN;

    // this lane's DMA slot: row 32 j + 8 wave + (lane >> 3) of piece j, LDS slot lane & 7 holding
    // source slot src (chunk kc of the step, plane offset pl for the split mode)
    const int src = (lane & 7) ^ (((lane >> 4) + 4 * (wave & 1)) & 7);
    const int kc = MODE == 1 ? (src & 3) : src;
    const int pl = MODE == 1 ? (src >> 2) * 16 : 0;
    const int ics = p.in_cstride ? p.in_cstride : p.Cin;
    const int64_t pixb = (int64_t)ics * C::EB;
    const int Cin8 = p.Cin >> 3, K8 = p.K >> 3;
    const char* in = (const char*)p.in;
    const char* wt = (const char*)p.w;
    const char* zero = (const char*)p.zero;
    // A rows: window origin (ih0, iw0) and its pixel address (outside the input for padded
    // rows: only dereferenced for in-bounds taps); rows past M never pass the bounds test
    int64_t abase[PA];
    int aih[PA], aiw[PA];
#pragma unroll
    for (int j = 0; j < PA; j++) {
        const int64_t m = m0 + 32 * j + 8 * wave + (lane >> 3);
        if (m < p.M) {
            const int ow = (int)(m % p.OW);
            const int64_t q = m / p.OW;
            const int oh = (int)(q % p.OH);
            const int64_t n = q / p.OH;
            aih[j] = oh * p.sh - p.ph;
            aiw[j] = ow * p.sw - p.pw;
            abase[j] = ((n * p.H + aih[j]) * p.W + aiw[j]) * pixb + pl;
        } else {
            aih[j] = -(1 << 29);
            aiw[j] = 0;
            abase[j] = 0;
        }
    }
    int64_t bbase[PB];
#pragma unroll
    for (int j = 0; j < PB; j++) {
        const int n = min(n0 + 32 * j + 8 * wave + (lane >> 3), p.Cout - 1);
        bbase[j] = (int64_t)n * p.K * C::EB + pl;
    }
    const int KT = (p.K + C::KS - 1) / C::KS;
    const int kt0 = tail ? (int)((int64_t)slice * KT / p.tail_split) : 0;
    const int kt1 = tail ? (int)((int64_t)(slice + 1) * KT / p.tail_split) : KT;
    // the lane's chunk c = (kh, kw, cc): k = 8 c = (kh * KW + kw) * Cin + 8 cc
    int c = kt0 * C::CPS + kc;
    int tap = c / Cin8, cc = c - tap * Cin8;
    int kh = tap / p.KW, kw = tap - kh * p.KW;
    const bool chk = p.ph | p.pw;  // padded windows: bounds-test every tap
    auto issue = [&](int s) {
        char* base = smem + s * C::ST;
        const bool kv = c < K8;
        const int64_t toff = ((int64_t)kh * p.W + kw) * pixb + cc * C::CB;
#pragma unroll
        for (int j = 0; j < PA; j++) {
            bool ok = kv && aih[j] + kh >= 0;
            if (chk) ok = ok && aih[j] + kh < p.H && (unsigned)(aiw[j] + kw) < (unsigned)p.W;
            const char* g = ok ? in + abase[j] + toff : zero;
            __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                             (void __attribute__((address_space(3)))*)(base + (wave + 4 * j) * 1024), 16,
                                             0, 0);
        }
#pragma unroll
        for (int j = 0; j < PB; j++) {
            const char* g = kv ? wt + bbase[j] + (int64_t)c * C::CB : zero;
            __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)g,
                                             (void __attribute__((address_space(3)))*)(base + C::A_ST + (wave + 4 * j) * 1024),
                                             16, 0, 0);
        }
    };
    auto advance = [&]() {
        c += C::CPS;
        cc += C::CPS;
        while (cc >= Cin8) {
            cc -= Cin8;
            if (++kw == p.KW) {
                kw = 0;
                kh++;
            }
        }
    };

    f4 acc[FM][FN], accx[MODE == 1 ? FM : 1][MODE == 1 ? FN : 1];
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    if constexpr (MODE == 1) {
#pragma unroll
        for (int i = 0; i < FM; i++)
#pragma unroll
            for (int j = 0; j < FN; j++) accx[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    }
    // fragment reads: row lane & 15 of a 16-row block, slot (lane >> 4) (plane 0 / k 0..31) and
    // 4 + (lane >> 4) (plane 1 / k 32..63), swizzled by (row >> 1) & 7
    const int hsw = (lane & 15) >> 1;
    const int o0 = (lane & 15) * RB + (((lane >> 4) ^ hsw) << 4);
    const int o1 = (lane & 15) * RB + (((4 + (lane >> 4)) ^ hsw) << 4);

    constexpr int NS = C::NS, PPS = PA + PB;  // DMA instructions per wave and stage
    static_assert(NS >= 2 && NS <= 4, "stages");
    // prologue: steps kt0 .. kt0 + NS - 2 in flight
    int issued = kt0;
#pragma unroll
    for (int s = 0; s < NS - 1; s++)
        if (issued < kt1) {
            if (s) advance();
            issue(s);
            issued++;
        }
    for (int kt = kt0; kt < kt1; kt++) {
        // this wave's pieces of step kt have landed (the steps issued after it may still be in
        // flight: counted vmcnt); after the barrier every wave's have, and every wave is done
        // reading the stage the next DMA overwrites (step kt - 1's)
        const int ahead = issued - kt - 1;
        if (NS >= 4 && ahead >= 2)
            wait_vm_barrier<(NS >= 4 ? 2 * PPS : 0)>();
        else if (NS >= 3 && ahead >= 1)
            wait_vm_barrier<(NS >= 3 ? PPS : 0)>();
        else
            wait_vm_barrier<0>();
        const int sb = (kt - kt0) % NS;
        if (issued < kt1) {
            advance();
            issue((issued - kt0) % NS);
            issued++;
        }
        const char* As = smem + sb * C::ST + wm * C::WM * RB;
        const char* Bs = smem + sb * C::ST + C::A_ST + wn * C::WN * RB;
        if constexpr (MODE == 1) {
            h8 b0[FN], b1[FN];
#pragma unroll
            for (int j = 0; j < FN; j++) {
                b0[j] = *(const h8*)(Bs + j * 16 * RB + o0);
                b1[j] = *(const h8*)(Bs + j * 16 * RB + o1);
            }
#pragma unroll
            for (int i = 0; i < FM; i++) {
                const h8 a0 = *(const h8*)(As + i * 16 * RB + o0);
                const h8 a1 = *(const h8*)(As + i * 16 * RB + o1);
#pragma unroll
                for (int j = 0; j < FN; j++) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b0[j], acc[i][j], 0, 0, 0);
                    accx[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b1[j], accx[i][j], 0, 0, 0);
                    accx[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b0[j], accx[i][j], 0, 0, 0);
                }
            }
        } else {
            bf16x8 b0[FN], b1[FN];
#pragma unroll
            for (int j = 0; j < FN; j++) {
                b0[j] = *(const bf16x8*)(Bs + j * 16 * RB + o0);
                b1[j] = *(const bf16x8*)(Bs + j * 16 * RB + o1);
            }
#pragma unroll
            for (int i = 0; i < FM; i++) {
                const bf16x8 a0 = *(const bf16x8*)(As + i * 16 * RB + o0);
                const bf16x8 a1 = *(const bf16x8*)(As + i * 16 * RB + o1);
#pragma unroll
                for (int j = 0; j < FN; j++) {
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a0, b0[j], acc[i][j], 0, 0, 0);
                    acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a1, b1[j], acc[i][j], 0, 0, 0);
                }
            }
        }
    }
    if constexpr (MODE == 1) {
#pragma unroll
        for (int i = 0; i < FM; i++)
#pragma unroll
            for (int j = 0; j < FN; j++) acc[i][j] = acc[i][j] + accx[i][j] * 0.00048828125f;
    }
    __syncthreads();  // no DMA outstanding; every wave is done with the stages
    if (tail) {
        // K slice of a tail tile: fp32 partial in fragment order (coalesced 16-B stores)
        f4* slab = (f4*)(p.ws + ((int64_t)(t - p.dp_tiles) * p.tail_split + slice) * (BM * BN));
#pragma unroll
        for (int i = 0; i < FM; i++)
#pragma unroll
            for (int j = 0; j < FN; j++) slab[((wave * FM + i) * FN + j) * 64 + lane] = acc[i][j];
        return;
    }
    float* E = (float*)smem;
#pragma unroll
    for (int j = 0; j < FN; j++)
#pragma unroll
        for (int i = 0; i < FM; i++)
#pragma unroll
            for (int q = 0; q < 4; q++)
                E[(wm * C::WM + i * 16 + 4 * (lane >> 4) + q) * C::LDE + wn * C::WN + j * 16 + (lane & 15)] = acc[i][j][q];
    __syncthreads();
    dma_epilogue<T, BN>(p, E, BM, m0, n0);
}

// ---------------------------------------------------------------- span mode (split pairs)
// Stride-1 unpadded convs (MTCNN RNet / ONet 3x3 on the candidate maps): the input pixels an M
// tile reads over all KH x KW taps form ONE contiguous run of the NHWC input -- output m = (n, oh,
// ow) reads idx(m) + kh W + kw with idx(m) = (n H + oh) W + ow -- so the tile's A operand is that
// run ("span": <= SPAN pixels x Cin = 32 Q channels of split pairs), copied into LDS once per tile
// by contiguous DMA, and every k-step's A fragment row is read from it at the lane's row offset
// idx(m) - idx(m0) + kh W + kw.  The implicit-GEMM gather fetched each input piece once per tap
// (9x for 3x3); here the tile's A traffic is its span.  B (weights) streams per k-step through NS
// LDS stages as in k_conv_dma.  Span rows are 128 Q bytes (a pixel's 8 Q logical 16-B slots: per
// 32-channel group [x0 of 4 chunks | x1 of 4 chunks] as in MODE 1), swizzled by a key of the
// pixel (n, y, x) in OUTPUT-linear coordinates, v = n OH OW + y OW + x: the 16 rows of a fragment
// read pixels with 16 consecutive v for every tap (v = m + kh OW + kw), while their span rows jump
// at output-row and image wraps (by an odd count for valid convs: KW - 1 + 1 and the image tail).
// Q = 1: physical slot = ls ^ span_key(v); Q = 2: slot over the whole 256-B row = (8 g + ls) ^
// span_key16(v) -- conflict-free for ds_read_b128's lane groups (span_key).
// k order (tap-major, then channel) and MFMA chains are k_conv_dma MODE 1's: the same bits when
// that kernel does not split K.
// a / d for 0 <= a < 2^22 and small d through the float reciprocal inv = 1 / d, corrected to the
// exact quotient (the span kernels' per-lane index math: ~6 VALU instead of an integer division)
__device__ inline int qdiv(int a, int d, float inv) {
    int q = (int)(((float)a + 0.5f) * inv);
    q -= q * d > a;
    q += (q + 1) * d <= a;
    return q;
}

// span-row swizzle keys of a pixel with output-linear index v (the 16 rows of a fragment read 16
// consecutive v under every tap, rows of alternating parity).  ds_read_b128 serves its 64 lanes in
// four 16-lane groups, e.g. {0-3, 12-15, 20-27}: rows 0-3 and 12-15 at chunk a, rows 4-11 at
// chunk a + 1.  With 128-B rows (bank half = row parity) a group is conflict-free iff, per parity
// class, the slots chunk ^ key are distinct; key = v & 6 gives rows u, u + 8 (same key, same
// parity) chunks a, a + 1 for every alignment of the 16 keys, so it is.  256-B rows (Q = 2) put the
// parity bit into slot bit 3 instead.  (Searched exhaustively; (v >> 1) & 7 conflicts for odd-
// aligned keys.)
__device__ inline int span_key(int v) { return v & 6; }
__device__ inline int span_key16(int v) { return (v & 6) | ((v & 1) << 3); }

template <int Q, int BM, int BN, int WGM, int SPAN, int OCC, int NS>
struct SCfg {
    static constexpr int WGN = 4 / WGM, WM = BM / WGM, WN = BN / WGN, FM = WM / 16, FN = WN / 16;
    static constexpr int RBA = 128 * Q, A_BYTES = SPAN * RBA, B_ST = BN * 128, LDE = BN + 4;
    static constexpr int SM0 = A_BYTES + NS * B_ST;
    static constexpr int SM = SM0 > BM * LDE * 4 ? SM0 : BM * LDE * 4;
    static constexpr int PB = BN / 32;  // 1-KB B pieces per wave and stage
    static_assert(SPAN % 8 == 0 && FM >= 1 && FN >= 1 && NS >= 2 && NS <= 3 && SM * OCC <= 160 * 1024, "span tile");
};

// largest span (input pixels) of any BM-row tile of this conv; tiles start at multiples of BM, so
// their offsets within an image repeat after OH*OW tiles
int64_t conv_span_max(const ConvParams& p, int BM) {
    const int64_t OHW = (int64_t)p.OH * p.OW, HW = (int64_t)p.H * p.W;
    auto idx = [&](int64_t m) {
        const int64_t n = m / OHW, r = m - n * OHW, oh = r / p.OW;
        return n * HW + oh * p.W + (r - oh * p.OW);
    };
    const int64_t T = (p.M + BM - 1) / BM;
    int64_t mx = 0;
    for (int64_t t = 0; t < std::min<int64_t>(T, OHW + 1); t++) {
        const int64_t m0 = t * BM, m1 = std::min<int64_t>(m0 + BM, p.M) - 1;
        mx = std::max<int64_t>(mx, idx(m1) - idx(m0) + (int64_t)(p.KH - 1) * p.W + p.KW);
    }
    if (T > OHW + 1) {  // the last (partial) tile
        const int64_t m0 = (T - 1) * BM;
        mx = std::max<int64_t>(mx, idx(p.M - 1) - idx(m0) + (int64_t)(p.KH - 1) * p.W + p.KW);
    }
    return mx;
}

template <int Q, int BM, int BN, int WGM, int SPAN, int OCC, int NS>
__global__ __launch_bounds__(256, OCC) void k_conv_span(ConvParams p) {
    using C = SCfg<Q, BM, BN, WGM, SPAN, OCC, NS>;
    constexpr int FM = C::FM, FN = C::FN, PB = C::PB, RBA = C::RBA;
    __shared__ __attribute__((aligned(16))) char smem[C::SM];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / C::WGN, wn = wave % C::WGN;
    int t, slice, tile_m, tile_n;
    bool tail;
    work_item(p, blockIdx.x, t, slice, tail);  // every tile whole (dp_tiles = all)
    tile_of(p, t, tile_m, tile_n);
    const int64_t m0 = (int64_t)tile_m * BM;
    const int n0 = tile_n * BN;
    const int64_t mlast = min(m0 + BM, p.M) - 1;
    const int OHW = p.OH * p.OW, HW = p.H * p.W;
    const float iOHW = 1.f / OHW, iOW = 1.f / p.OW, iHW = 1.f / HW, iW = 1.f / p.W;
    // the tile's first output (n0i, oh0, ow0) once; lanes work relative to it: output m of the
    // tile (d = m - m0 < BM) has its input pixel at rel(d) from P0 = (n0i H + oh0) W + ow0
    const int64_t n0i = m0 / OHW;
    const int r0 = (int)(m0 - n0i * OHW), oh0 = qdiv(r0, p.OW, iOW), base0 = oh0 * p.W + (r0 - oh0 * p.OW);
    auto rel = [&](int d) -> int {
        const int mr = r0 + d, dn = qdiv(mr, OHW, iOHW), r = mr - dn * OHW, oh = qdiv(r, p.OW, iOW);
        return dn * HW + oh * p.W + (r - oh * p.OW) - base0;
    };
    const int64_t P0 = n0i * HW + base0, npix = (int64_t)p.N * HW;
    const int span = rel((int)(mlast - m0)) + (p.KH - 1) * p.W + p.KW;  // <= SPAN (host-checked)
    const int key0 = (int)((n0i * OHW) & 15);
    const char* in = (const char*)p.in;
    const char* wt = (const char*)p.w;
    const char* zero = (const char*)p.zero;
    // A span: 1-KB DMA pieces dealt round-robin to the waves (lane-linear LDS destination)
    const int nA = (span * RBA + 1023) >> 10;
    for (int j = wave; j < nA; j += 4) {
        const int off = j * 1024 + lane * 16;
        const int row = off / RBA;
        const int64_t pix = P0 + row;
        // the pixel's swizzle key: v = n OH OW + y OW + x (mod 16) of its (n, y, x)
        const int loc = base0 + row, dn = qdiv(loc, HW, iHW), rem = loc - dn * HW, y = qdiv(rem, p.W, iW);
        const int v = key0 + dn * OHW + y * p.OW + (rem - y * p.W);
        int g, ls;
        if (Q == 1) {
            g = 0;
            ls = ((off >> 4) & 7) ^ span_key(v);
        } else {
            const int lg = ((off >> 4) & 15) ^ span_key16(v);
            g = lg >> 3;
            ls = lg & 7;
        }
        const char* src =
            row < span && pix < npix ? in + pix * (128 * Q) + g * 128 + (ls & 3) * 32 + (ls >> 2) * 16 : zero;
        __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                         (void __attribute__((address_space(3)))*)(smem + off), 16, 0, 0);
    }
    // B: as k_conv_dma MODE 1 (row 32 j + 8 wave + (lane >> 3) of piece j, swizzled slot)
    const int bsrc = (lane & 7) ^ (((lane >> 4) + 4 * (wave & 1)) & 7);
    const int bkc = bsrc & 3, bpl = (bsrc >> 2) * 16;
    int64_t bbase[PB];
#pragma unroll
    for (int j = 0; j < PB; j++) {
        const int n = min(n0 + 32 * j + 8 * wave + (lane >> 3), p.Cout - 1);
        bbase[j] = (int64_t)n * p.K * 4 + bpl + bkc * 32;
    }
    char* Bst = smem + C::A_BYTES;
    auto issueB = [&](int kt, int s) {
#pragma unroll
        for (int j = 0; j < PB; j++)
            __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(wt + bbase[j] + (int64_t)kt * 128),
                                             (void __attribute__((address_space(3)))*)(Bst + s * C::B_ST + (wave + 4 * j) * 1024),
                                             16, 0, 0);
    };
    // the lane's A rows (span-relative) of its FM fragments; rows past M repeat the last row
    int arow[FM], akey[FM];
#pragma unroll
    for (int i = 0; i < FM; i++) {
        const int d = (int)min((int64_t)(wm * C::WM + i * 16 + (lane & 15)), mlast - m0);
        arow[i] = rel(d);
        akey[i] = (int)((m0 + d) & 15);  // + kh OW + kw: the swizzle key of the pixel a tap reads
    }
    f4 acc[FM][FN], accx[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = accx[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    const int hsw = (lane & 15) >> 1;
    const int o0 = (lane & 15) * 128 + (((lane >> 4) ^ hsw) << 4);
    const int o1 = (lane & 15) * 128 + (((4 + (lane >> 4)) ^ hsw) << 4);
    const int KT = p.K >> 5;
    // prologue: B steps 0 .. NS - 2 in flight behind the span
    int issued = 0;
#pragma unroll
    for (int s = 0; s < NS - 1; s++)
        if (issued < KT) {
            issueB(issued, issued % NS);
            issued++;
        }
    int kh = 0, kw = 0, g = 0;
    for (int kt = 0; kt < KT; kt++) {
        // this wave's B step kt (and the span, issued first) landed: counted vmcnt leaves the
        // later steps in flight; after the barrier for every wave, and the stage the next issue
        // overwrites (step kt - 1's) is free
        if (NS >= 3 && issued - kt - 1 >= 1)
            wait_vm_barrier<(NS >= 3 ? PB : 0)>();
        else
            wait_vm_barrier<0>();
        if (issued < KT) {
            issueB(issued, issued % NS);
            issued++;
        }
        const char* Bs = Bst + (kt % NS) * C::B_ST + wn * C::WN * 128;
        h8 b0[FN], b1[FN];
#pragma unroll
        for (int j = 0; j < FN; j++) {
            b0[j] = *(const h8*)(Bs + j * 16 * 128 + o0);
            b1[j] = *(const h8*)(Bs + j * 16 * 128 + o1);
        }
        const int toff = kh * p.W + kw, tkey = kh * p.OW + kw;
#pragma unroll
        for (int i = 0; i < FM; i++) {
            const int v = akey[i] + tkey;
            const char* Ar = smem + (arow[i] + toff) * RBA;
            int s0, s1;
            if (Q == 1) {
                s0 = (lane >> 4) ^ span_key(v);
                s1 = (4 + (lane >> 4)) ^ span_key(v);
            } else {
                s0 = (8 * g + (lane >> 4)) ^ span_key16(v);
                s1 = (8 * g + 4 + (lane >> 4)) ^ span_key16(v);
            }
            const h8 a0 = *(const h8*)(Ar + (s0 << 4));
            const h8 a1 = *(const h8*)(Ar + (s1 << 4));
#pragma unroll
            for (int j = 0; j < FN; j++) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b0[j], acc[i][j], 0, 0, 0);
                accx[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b1[j], accx[i][j], 0, 0, 0);
                accx[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b0[j], accx[i][j], 0, 0, 0);
            }
        }
        if (++g == Q) {
            g = 0;
            if (++kw == p.KW) {
                kw = 0;
                kh++;
            }
        }
    }
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = acc[i][j] + accx[i][j] * 0.00048828125f;
    __syncthreads();  // no DMA outstanding; every wave is done with the span and the stages
    float* E = (float*)smem;
#pragma unroll
    for (int j = 0; j < FN; j++)
#pragma unroll
        for (int i = 0; i < FM; i++)
#pragma unroll
            for (int q = 0; q < 4; q++)
                E[(wm * C::WM + i * 16 + 4 * (lane >> 4) + q) * C::LDE + wn * C::WN + j * 16 + (lane & 15)] = acc[i][j][q];
    __syncthreads();
    dma_epilogue<float, BN>(p, E, BM, m0, n0);
}

// ---------------------------------------------------------------- span mode + fused max-pool
// The span kernel for a conv followed by MaxPool2d(pk, ps, ceil) (RNet conv2 -> pool1, ONet
// conv2 -> pool1; mtcnn.py:41-121): tiles are aligned to the pool instead of to BM rows -- a tile
// is `cg` whole candidates (parts = 1) or one of `parts` row bands of one candidate, a band being
// the conv rows its pool rows read (ONet: pool rows 0-4 <- conv rows 0-10, 5-9 <- 10-20; the
// shared row is computed twice).  The conv tile (bias + PReLU applied) stays in LDS and the
// workgroup writes only the pooled map, in the split-pair layout with the range flag: the conv
// output never goes to HBM and the separate pool launch is gone.  M-row r of a tile = (candidate
// cl, band row y, column x), r = (cl RP + y) OW + x; its span row = cl H W + y W + x (+ kh W + kw
// per tap) relative to the band's first input pixel; the swizzle key is r + kh OW + kw, the
// k_conv_span argument (row jumps at x / candidate wraps are KW and KH W - OW + 1: odd).
struct SpanPool {
    int k, s, POH, POW;  // pool window, stride, pooled map
    int cg, parts;       // candidates per tile (parts = 1) / bands per candidate (cg = 1)
    int RP, PH2;         // conv rows per band (max), pool rows per band
    void* out;           // pooled map [N][POH][POW][Cout] split pairs
};

template <int BM, int BN, int SPAN, int NS>
struct SPCfg {
    static constexpr int WM = BM / 4, FM = WM / 16, FN = BN / 16;  // 4 waves x (WM rows, all BN cols)
    static constexpr int A_BYTES = SPAN * 128, B_ST = BN * 128, LDE = BN + 4;
    static constexpr int SM0 = A_BYTES + NS * B_ST;
    static constexpr int SM = SM0 > BM * LDE * 4 ? SM0 : BM * LDE * 4;
    static constexpr int PB = BN / 32;
    static_assert(SPAN % 8 == 0 && FM >= 1 && NS >= 2 && NS <= 4 && SM * 2 <= 160 * 1024, "span-pool tile");
};

// NS B stages: NS - 1 weight k-steps in flight; FNU: the 16-column fragments computed (RNet's
// 48 output channels: 3 of the tile's 4 -- the weight rows past Cout are staged but never used)
template <int BM, int BN, int SPAN, int NS, int FNU = BN / 16>
__global__ __launch_bounds__(256, 2) void k_conv_span_pool(ConvParams p, SpanPool sp) {
    using C = SPCfg<BM, BN, SPAN, NS>;
    static_assert(FNU >= 1 && FNU <= C::FN, "fragments used");
    constexpr int FM = C::FM, FN = FNU, PB = C::PB;
    __shared__ __attribute__((aligned(16))) char smem[C::SM];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int t = blockIdx.x;
    const int HW = p.H * p.W;
    // the tile: candidates n0 .. n0 + ncand - 1, conv rows oy0 .. oy0 + rp - 1, pool rows py0 .. py1 - 1
    const int n0 = sp.parts == 1 ? t * sp.cg : t / sp.parts, part = sp.parts == 1 ? 0 : t % sp.parts;
    const int ncand = min(sp.cg, p.N - n0);
    const int py0 = part * sp.PH2, py1 = min(sp.POH, py0 + sp.PH2);
    const int oy0 = py0 * sp.s, rp = min(p.OH, (py1 - 1) * sp.s + sp.k) - oy0;
    const int rows = ncand * rp * p.OW;  // valid M rows of the tile (<= BM, host-checked)
    const int64_t P0 = (int64_t)n0 * HW + (int64_t)oy0 * p.W;
    const int RPW = rp * p.OW;
    const float iHW = 1.f / HW, iW = 1.f / p.W, iOW = 1.f / p.OW, iRPW = 1.f / RPW;
    const int span = (ncand - 1) * HW + (rp + p.KH - 1) * p.W;  // <= SPAN (host-checked)
    const char* in = (const char*)p.in;
    const char* wt = (const char*)p.w;
    const char* zero = (const char*)p.zero;
    // span DMA: pixel L = (cl, y, x) of the band, key v = (cl rp + y) OW + x
    const int nA = (span * 128 + 1023) >> 10;
    for (int j = wave; j < nA; j += 4) {
        const int off = j * 1024 + lane * 16, row = off >> 7;
        const int cl = qdiv(row, HW, iHW), rem = row - cl * HW, y = qdiv(rem, p.W, iW), x = rem - y * p.W;
        const int v = (cl * rp + y) * p.OW + x;
        const int ls = ((off >> 4) & 7) ^ span_key(v);
        const char* src = row < span ? in + (P0 + row) * 128 + (ls & 3) * 32 + (ls >> 2) * 16 : zero;
        __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)src,
                                         (void __attribute__((address_space(3)))*)(smem + off), 16, 0, 0);
    }
    const int bsrc = (lane & 7) ^ (((lane >> 4) + 4 * (wave & 1)) & 7);
    int64_t bbase[PB];
#pragma unroll
    for (int j = 0; j < PB; j++) {
        const int n = min(32 * j + 8 * wave + (lane >> 3), p.Cout - 1);
        bbase[j] = (int64_t)n * p.K * 4 + (bsrc >> 2) * 16 + (bsrc & 3) * 32;
    }
    char* Bst = smem + C::A_BYTES;
    auto issueB = [&](int kt, int s) {
#pragma unroll
        for (int j = 0; j < PB; j++)
            __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(wt + bbase[j] + (int64_t)kt * 128),
                                             (void __attribute__((address_space(3)))*)(Bst + s * C::B_ST + (wave + 4 * j) * 1024),
                                             16, 0, 0);
    };
    int arow[FM], akey[FM];
#pragma unroll
    for (int i = 0; i < FM; i++) {
        const int r = min(wave * C::WM + i * 16 + (lane & 15), rows - 1);
        const int cl = qdiv(r, RPW, iRPW), q = r - cl * RPW, y = qdiv(q, p.OW, iOW);
        arow[i] = cl * HW + y * p.W + (q - y * p.OW);
        akey[i] = r;
    }
    f4 acc[FM][FN], accx[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = accx[i][j] = f4{0.f, 0.f, 0.f, 0.f};
    const int hsw = (lane & 15) >> 1;
    const int o0 = (lane & 15) * 128 + (((lane >> 4) ^ hsw) << 4);
    const int o1 = (lane & 15) * 128 + (((4 + (lane >> 4)) ^ hsw) << 4);
    const int KT = p.K >> 5;
    int issued = 0;
#pragma unroll
    for (int s = 0; s < NS - 1; s++)
        if (issued < KT) {
            issueB(issued, issued % NS);
            issued++;
        }
    int kh = 0, kw = 0;
    for (int kt = 0; kt < KT; kt++) {
        // counted vmcnt: this wave's B step kt (and the span, issued first) landed, the later
        // steps may still be in flight; after the barrier for every wave, and step kt - 1's
        // stage (the next issue's) is free
        const int ahead = issued - kt - 1;
        if (NS >= 4 && ahead >= 2)
            wait_vm_barrier<(NS >= 4 ? 2 * PB : 0)>();
        else if (NS >= 3 && ahead >= 1)
            wait_vm_barrier<(NS >= 3 ? PB : 0)>();
        else
            wait_vm_barrier<0>();
        if (issued < KT) {
            issueB(issued, issued % NS);
            issued++;
        }
        const char* Bs = Bst + (kt % NS) * C::B_ST;
        h8 b0[FN], b1[FN];
#pragma unroll
        for (int j = 0; j < FN; j++) {
            b0[j] = *(const h8*)(Bs + j * 16 * 128 + o0);
            b1[j] = *(const h8*)(Bs + j * 16 * 128 + o1);
        }
        const int toff = kh * p.W + kw, tkey = kh * p.OW + kw;
#pragma unroll
        for (int i = 0; i < FM; i++) {
            const int sw = span_key(akey[i] + tkey);
            const char* Ar = smem + (arow[i] + toff) * 128;
            const h8 a0 = *(const h8*)(Ar + (((lane >> 4) ^ sw) << 4));
            const h8 a1 = *(const h8*)(Ar + (((4 + (lane >> 4)) ^ sw) << 4));
#pragma unroll
            for (int j = 0; j < FN; j++) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b0[j], acc[i][j], 0, 0, 0);
                accx[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b1[j], accx[i][j], 0, 0, 0);
                accx[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b0[j], accx[i][j], 0, 0, 0);
            }
        }
        if (++kw == p.KW) {
            kw = 0;
            kh++;
        }
    }
    __syncthreads();  // no DMA outstanding; the span and the stages are free for the tile image
    // conv epilogue into LDS: v = acc + 2^-11 accx, + bias, PReLU (conv_epilogue8's order)
    float* E = (float*)smem;
#pragma unroll
    for (int j = 0; j < FN; j++) {
        const int c = min(j * 16 + (lane & 15), p.Cout - 1);
        const float bb = p.bias ? p.bias[c] : 0.f, pa = p.prelu ? p.prelu[c] : 0.f;
#pragma unroll
        for (int i = 0; i < FM; i++)
#pragma unroll
            for (int q = 0; q < 4; q++) {
                float x = acc[i][j][q] + accx[i][j][q] * 0.00048828125f;
                if (p.bias) x = x + bb;
                if (p.prelu) x = x > 0.f ? x : pa * x;
                E[(wave * C::WM + i * 16 + 4 * (lane >> 4) + q) * C::LDE + j * 16 + (lane & 15)] = x;
            }
    }
    __syncthreads();
    // max-pool of the band (windows clipped at the conv map's last row / column, ceil mode) ->
    // split pairs, 8 channels per item
    const int C8 = p.Cout >> 3, npy = py1 - py0;
    const int items = ncand * npy * sp.POW * C8;
    const float iC8 = 1.f / C8, iPOW = 1.f / sp.POW, iNPY = 1.f / npy;
    bool bad = false;
    for (int it = tid; it < items; it += 256) {
        const int q = qdiv(it, C8, iC8), c8 = it - q * C8, q2 = qdiv(q, sp.POW, iPOW), px = q - q2 * sp.POW;
        const int cl = qdiv(q2, npy, iNPY), pyl = q2 - cl * npy;
        const int py = py0 + pyl;
        float m[8];
#pragma unroll
        for (int e = 0; e < 8; e++) m[e] = -3.402823466e38f;
        for (int dy = 0; dy < sp.k; dy++) {
            const int y = py * sp.s + dy;
            if (y >= p.OH) break;
            for (int dx = 0; dx < sp.k; dx++) {
                const int x = px * sp.s + dx;
                if (x >= p.OW) break;
                const float* e = E + ((cl * rp + (y - oy0)) * p.OW + x) * C::LDE + 8 * c8;
                const f4 lo = *(const f4*)e, hi = *(const f4*)(e + 4);
#pragma unroll
                for (int u = 0; u < 4; u++) {
                    m[u] = fmaxf(m[u], lo[u]);
                    m[4 + u] = fmaxf(m[4 + u], hi[u]);
                }
            }
        }
        char* orow = (char*)sp.out + (((int64_t)(n0 + cl) * sp.POH + py) * sp.POW + px) * (int64_t)p.Cout * 4;
        sp_store4(orow, 8 * c8, m[0], m[1], m[2], m[3], bad);
        sp_store4(orow, 8 * c8 + 4, m[4], m[5], m[6], m[7], bad);
    }
    if (p.ovf && __ballot(bad) && lane == 0) atomicOr(p.ovf, 1);
}

// ---------------------------------------------------------------- MODE 2: bf16x3 (fp32-grade)
// Operands in the split-triple layout (conv_dev.hpp: x = b0 + b1 + b2, three bf16 terms of 8
// significant bits each), so every fp32 product is x w = b0 w0 + [b0 w1 + b1 w0 + b0 w2 + b1 w1 +
// b2 w0] up to terms of 2^-24 relative: six v_mfma_f32_16x16x32_bf16 per 32-deep step and
// fragment pair (96 cycles) instead of eight v_mfma_f32_16x16x4_f32 (256), with fp32's exponent
// range (YOLO's Darknet activations reach 1.5e5 with the synthetic weights: beyond the fp16 split).
// LDS image per stage: three planes of A rows then three planes of B rows, 64-B rows (one
// 32-deep step of one plane: 4 chunks), 16-B slot s of row r holding chunk s ^ f((r >> 2) & 3) with
// f(x) = (4 - x) & 3 -- conflict-free for the ds_read_b128 fragment reads (rows lane & 15, chunk
// lane >> 4); a DMA wave-instruction writes one plane's 16-row block (1 KB) lane-linearly.
template <int BM, int BN, int WGM>
struct D3Cfg {
    static constexpr int WGN = 4 / WGM, WM = BM / WGM, WN = BN / WGN, FM = WM / 16, FN = WN / 16;
    static constexpr int RB = 64, PLA = BM * RB, PLB = BN * RB, A_ST = 3 * PLA, ST = 3 * (PLA + PLB), LDE = BN + 4;
    static constexpr int SM = 2 * ST > BM * LDE * 4 ? 2 * ST : BM * LDE * 4;
    static constexpr int RA = BM / 64, RBN = BN / 64;  // 16-row blocks per wave (A, B)
    static_assert(BM % 64 == 0 && BN % 64 == 0 && FM >= 1 && FN >= 1 && SM * 2 <= 160 * 1024, "bf16x3 tile");
};

__device__ inline int s3_swz(int r) { return (4 - ((r >> 2) & 3)) & 3; }

template <int BM, int BN, int WGM>
__global__ __launch_bounds__(256, 2) void k_conv_dma3(ConvParams p) {
    using C = D3Cfg<BM, BN, WGM>;
    constexpr int FM = C::FM, FN = C::FN, RB = C::RB, RA = C::RA, RBN = C::RBN;
    __shared__ __attribute__((aligned(16))) char smem[C::SM];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave / C::WGN, wn = wave % C::WGN;
    int t, slice, tile_m, tile_n;
    bool tail;
    work_item(p, blockIdx.x, t, slice, tail);
    tile_of(p, t, tile_m, tile_n);
    const int64_t m0 = (int64_t)tile_m * BM;
    const int n0 = tile_n * BN;
    // DMA: lane L of a 16-row block writes row L >> 2, slot L & 3, which holds chunk
    // kc = (L & 3) ^ f((L >> 4) & 3) of the step (the same for every block of the lane)
    const int kc = (lane & 3) ^ s3_swz(lane >> 2);
    const int ics = p.in_cstride ? p.in_cstride : p.Cin;
    const int64_t pixb = (int64_t)ics * 6;
    const int Cin8 = p.Cin >> 3, K8 = p.K >> 3;
    const char* in = (const char*)p.in;
    const char* wt = (const char*)p.w;
    const char* zero = (const char*)p.zero;
    int64_t abase[RA];
    int aih[RA], aiw[RA];
#pragma unroll
    for (int j = 0; j < RA; j++) {
        const int64_t m = m0 + 16 * (wave + 4 * j) + (lane >> 2);
        if (m < p.M) {
            const int ow = (int)(m % p.OW);
            const int64_t q = m / p.OW;
            const int oh = (int)(q % p.OH);
            const int64_t n = q / p.OH;
            aih[j] = oh * p.sh - p.ph;
            aiw[j] = ow * p.sw - p.pw;
            abase[j] = ((n * p.H + aih[j]) * p.W + aiw[j]) * pixb;
        } else {
            aih[j] = -(1 << 29);
            aiw[j] = 0;
            abase[j] = 0;
        }
    }
    int64_t bbase[RBN];
#pragma unroll
    for (int j = 0; j < RBN; j++) {
        const int n = min(n0 + 16 * (wave + 4 * j) + (lane >> 2), p.Cout - 1);
        bbase[j] = (int64_t)n * K8 * 48;
    }
    const int KT = (p.K + 31) / 32;
    const int kt0 = tail ? (int)((int64_t)slice * KT / p.tail_split) : 0;
    const int kt1 = tail ? (int)((int64_t)(slice + 1) * KT / p.tail_split) : KT;
    int c = kt0 * 4 + kc;
    int tap = c / Cin8, cc = c - tap * Cin8;
    int kh = tap / p.KW, kw = tap - kh * p.KW;
    const bool chk = p.ph | p.pw;
    auto issue = [&](int s) {
        char* base = smem + s * C::ST;
        const bool kv = c < K8;
        const int64_t toff = ((int64_t)kh * p.W + kw) * pixb + cc * 48;
#pragma unroll
        for (int j = 0; j < RA; j++) {
            bool ok = kv && aih[j] + kh >= 0;
            if (chk) ok = ok && aih[j] + kh < p.H && (unsigned)(aiw[j] + kw) < (unsigned)p.W;
            const char* g = ok ? in + abase[j] + toff : zero;
#pragma unroll
            for (int pl = 0; pl < 3; pl++)
                __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(ok ? g + 16 * pl : zero),
                                                 (void __attribute__((address_space(3)))*)(base + pl * C::PLA +
                                                                                           (wave + 4 * j) * 1024),
                                                 16, 0, 0);
        }
#pragma unroll
        for (int j = 0; j < RBN; j++) {
            const char* g = wt + bbase[j] + (int64_t)c * 48;
#pragma unroll
            for (int pl = 0; pl < 3; pl++)
                __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(kv ? g + 16 * pl : zero),
                                                 (void __attribute__((address_space(3)))*)(base + C::A_ST + pl * C::PLB +
                                                                                           (wave + 4 * j) * 1024),
                                                 16, 0, 0);
        }
    };
    auto advance = [&]() {
        c += 4;
        cc += 4;
        while (cc >= Cin8) {
            cc -= Cin8;
            if (++kw == p.KW) {
                kw = 0;
                kh++;
            }
        }
    };
    f4 acc[FM][FN], accx[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) {
            acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
            accx[i][j] = f4{0.f, 0.f, 0.f, 0.f};
        }
    const int of = (lane & 15) * RB + (((lane >> 4) ^ s3_swz(lane & 15)) << 4);
    issue(0);
    for (int kt = kt0; kt < kt1; kt++) {
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        const int sb = (kt - kt0) & 1;
        if (kt + 1 < kt1) {
            advance();
            issue(sb ^ 1);
        }
        const char* As = smem + sb * C::ST + wm * C::WM * RB + of;
        const char* Bs = smem + sb * C::ST + C::A_ST + wn * C::WN * RB + of;
        bf16x8 b[FN][3];
#pragma unroll
        for (int j = 0; j < FN; j++)
#pragma unroll
            for (int pl = 0; pl < 3; pl++) b[j][pl] = *(const bf16x8*)(Bs + pl * C::PLB + j * 16 * RB);
#pragma unroll
        for (int i = 0; i < FM; i++) {
            bf16x8 a[3];
#pragma unroll
            for (int pl = 0; pl < 3; pl++) a[pl] = *(const bf16x8*)(As + pl * C::PLA + i * 16 * RB);
#pragma unroll
            for (int j = 0; j < FN; j++) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[j][0], acc[i][j], 0, 0, 0);
                accx[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[j][1], accx[i][j], 0, 0, 0);
                accx[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[j][0], accx[i][j], 0, 0, 0);
                accx[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[0], b[j][2], accx[i][j], 0, 0, 0);
                accx[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[1], b[j][1], accx[i][j], 0, 0, 0);
                accx[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a[2], b[j][0], accx[i][j], 0, 0, 0);
            }
        }
    }
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = acc[i][j] + accx[i][j];
    __syncthreads();
    if (tail) {
        f4* slab = (f4*)(p.ws + ((int64_t)(t - p.dp_tiles) * p.tail_split + slice) * (BM * BN));
#pragma unroll
        for (int i = 0; i < FM; i++)
#pragma unroll
            for (int j = 0; j < FN; j++) slab[((wave * FM + i) * FN + j) * 64 + lane] = acc[i][j];
        return;
    }
    float* E = (float*)smem;
#pragma unroll
    for (int j = 0; j < FN; j++)
#pragma unroll
        for (int i = 0; i < FM; i++)
#pragma unroll
            for (int q = 0; q < 4; q++)
                E[(wm * C::WM + i * 16 + 4 * (lane >> 4) + q) * C::LDE + wn * C::WN + j * 16 + (lane & 15)] = acc[i][j][q];
    __syncthreads();
    dma_epilogue<float, BN>(p, E, BM, m0, n0);
}

// tail tiles: one workgroup per (tile, 16-row block, 64-column half when BN = 128) sums the
// block's K slices in slice order (deterministic) into an LDS image, then the epilogue of those
// rows (one f4 of partial sums per thread)
template <int MODE, int BM, int BN, int WGM, int OCC, int NSTG>
__global__ __launch_bounds__(256) void k_conv_dma_tail(ConvParams p) {
    using C = DCfg<MODE, BM, BN, WGM, OCC, NSTG>;
    using T = typename std::conditional<MODE == 0, __bf16, float>::type;
    constexpr int NH = BN * 4 / 256 > 1 ? BN * 4 / 256 : 1;  // workgroups per 16-row block
    constexpr int NB = BM / 16 * NH, FM = C::FM, FN = C::FN, LDE = C::LDE;
    __shared__ __attribute__((aligned(16))) float E[16 * LDE];
    const int tid = threadIdx.x;
    const int tt = blockIdx.x / NB, rb = (blockIdx.x % NB) / NH, hpart = (blockIdx.x % NB) % NH;
    const int wm = rb / FM, i = rb % FM;
    int tile_m, tile_n;
    tile_of(p, p.dp_tiles + tt, tile_m, tile_n);
    const f4* s0 = (const f4*)(p.ws + (int64_t)tt * p.tail_split * (BM * BN));
    for (int f = tid + 256 * hpart; f < min(BN * 4, 256 * (hpart + 1)); f += 256) {  // (wn, j) x 64 lanes
        const int wn = f / (FN * 64), j = (f / 64) % FN, lane = f & 63;
        const int idx = (((wm * C::WGN + wn) * FM + i) * FN + j) * 64 + lane;
        f4 v = s0[idx];
        for (int z = 1; z < p.tail_split; z++) v = v + s0[(int64_t)z * (BM * BN / 4) + idx];
#pragma unroll
        for (int q = 0; q < 4; q++) E[(4 * (lane >> 4) + q) * LDE + wn * C::WN + j * 16 + (lane & 15)] = v[q];
    }
    __syncthreads();
    if constexpr (NH == 1) {
        dma_epilogue<T, BN>(p, E, 16, (int64_t)tile_m * BM + wm * C::WM + i * 16, tile_n * BN);
    } else {
        // this workgroup's columns: [256 hpart / 4, + 64) of the tile (E rows keep the tile's stride)
        dma_epilogue_cols<T, BN, 64>(p, E, 16, (int64_t)tile_m * BM + wm * C::WM + i * 16, tile_n * BN, 64 * hpart);
    }
}

// per-(device, stream) tail workspace: grows x1.5.  An outgrown buffer may still be read by
// kernels queued on its stream, so it is retired with an event recorded on that stream and
// freed at a later grow once the event has completed (freeing it at once would need a
// device-wide synchronisation that stalls the other lanes).  release_dma_ws(st) drops a
// stream's entry (vtf_release_stream).
namespace {
struct DmaWs {
    std::mutex mu;
    std::map<std::pair<int, hipStream_t>, std::pair<float*, size_t>> m;
    std::vector<std::pair<void*, hipEvent_t>> retired;
    void reap() {
        for (size_t i = 0; i < retired.size();) {
            if (hipEventQuery(retired[i].second) == hipSuccess) {
                (void)hipFree(retired[i].first);
                (void)hipEventDestroy(retired[i].second);
                retired[i] = retired.back();
                retired.pop_back();
            } else {
                i++;
            }
        }
    }
    void retire(void* p, hipStream_t st) {
        hipEvent_t ev;
        VTF_HIP(hipEventCreateWithFlags(&ev, hipEventDisableTiming));
        VTF_HIP(hipEventRecord(ev, st));
        retired.push_back({p, ev});
    }
};
DmaWs& dma_ws_state() {
    static DmaWs* s = new DmaWs();  // process lifetime (no destruction-order issues at exit)
    return *s;
}
}  // namespace

float* dma_ws(hipStream_t st, size_t bytes) {
    DmaWs& S = dma_ws_state();
    std::lock_guard<std::mutex> g(S.mu);
    auto& w = S.m[{stream_device(st), st}];
    if (w.second < bytes) {
        S.reap();
        if (w.first) S.retire(w.first, st);
        w.first = nullptr;
        w.second = 0;
        const size_t b = bytes + bytes / 2;
        VTF_HIP(hipMalloc((void**)&w.first, b));
        w.second = b;
    }
    return w.first;
}

void release_dma_ws_impl(hipStream_t st) {
    DmaWs& S = dma_ws_state();
    std::lock_guard<std::mutex> g(S.mu);
    auto it = S.m.find({stream_device(st), st});
    if (it != S.m.end()) {
        if (it->second.first) S.retire(it->second.first, st);
        S.m.erase(it);
    }
    S.reap();
}

// 16 zero bytes per device (the DMA source of padding, K-tail and M-tail pieces)
const void* zero_page(int dev) {
    static std::mutex mu;
    static std::map<int, void*> m;
    std::lock_guard<std::mutex> g(mu);
    void*& z = m[dev];
    if (!z) {
        VTF_HIP(hipMalloc(&z, 256));
        VTF_HIP(hipMemset(z, 0, 256));
    }
    return z;
}

int cu_count() {
    static int cus = [] {
        int dev = 0, n = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        return n;
    }();
    return cus;
}

int dma_group_m() {
    static int g = [] {
        const char* e = std::getenv("VTF_CONV_GROUP_M");
        return e ? std::atoi(e) : 8;
    }();
    return g;
}

template <int MODE, int BM, int BN, int WGM, int OCC = 2, int NSTG = 2>
void launch_dma_t(ConvParams p, hipStream_t st) {
    using C = DCfg<MODE, BM, BN, WGM, OCC, NSTG>;
    p.gx = (int)cdiv(p.M, BM);
    p.gy = (int)cdiv(p.Cout, BN);
    p.group_m = dma_group_m();
    p.zero = zero_page(stream_device(st));
    const int T = p.gx * p.gy, KT = (p.K + C::KS - 1) / C::KS;
    const int slots = OCC * cu_count();
    p.dp_tiles = T;
    p.tail_split = 1;
    p.split = 1;
    if ((MODE == 0 || p.split_fp32) && !splitk_disabled()) {
        if (T > slots) {
            // a last round of only a few tiles: split those along K over the free slots
            const int R = T % slots;
            const int S = R > 0 ? std::min(slots / R, KT / 4) : 0;
            if (R > 0 && R <= slots / 2 && S >= 2) {
                p.dp_tiles = T - R;
                p.tail_split = S;
            }
        } else {
            // less than one round: split every tile (>= 4 k-steps per slice)
            const int S = std::min(std::min(slots / T, KT / 4), 16);
            if (S >= 2) {
                p.dp_tiles = 0;
                p.tail_split = S;
            }
        }
    }
    const int nt = T - p.dp_tiles;
    p.ws = nt ? dma_ws(st, (size_t)nt * p.tail_split * BM * BN * 4) : nullptr;
    k_conv_dma<MODE, BM, BN, WGM, OCC, NSTG><<<(unsigned)(p.dp_tiles + nt * p.tail_split), 256, 0, st>>>(p);
    if (nt) k_conv_dma_tail<MODE, BM, BN, WGM, OCC, NSTG><<<(unsigned)(nt * (BM / 16) * (BN > 64 ? BN / 64 : 1)), 256, 0, st>>>(p);
}

template <int Q, int BM, int BN, int WGM, int SPAN, int OCC, int NS>
void launch_span_t(ConvParams p, hipStream_t st) {
    p.gx = (int)cdiv(p.M, BM);
    p.gy = (int)cdiv(p.Cout, BN);
    p.group_m = dma_group_m();
    p.zero = zero_page(stream_device(st));
    p.dp_tiles = p.gx * p.gy;
    p.tail_split = 1;
    p.split = 1;
    p.ws = nullptr;
    k_conv_span<Q, BM, BN, WGM, SPAN, OCC, NS><<<(unsigned)p.dp_tiles, 256, 0, st>>>(p);
}

// span-mode eligibility (split-pair, stride-1 unpadded convs of 32 / 64 input channels, odd KW
// (the swizzle pairs need odd row jumps), whose
// tiles' input runs fit the LDS span); env VTF_CONV_SPAN=0 keeps the implicit-GEMM gather
constexpr int SPAN_BM = 128, SPAN_ROWS = 240;
bool conv_span_ok(const ConvParams& p) {
    const char* e = std::getenv("VTF_CONV_SPAN");  // read per launch: tests A/B both paths in one process
    return (!e || std::atoi(e) != 0) && p.in_sp && !p.s3 && p.sh == 1 && p.sw == 1 && p.ph == 0 && p.pw == 0 &&
           (p.Cin == 32 || p.Cin == 64) && (p.in_cstride == 0 || p.in_cstride == p.Cin) && p.Cout <= 64 &&
           p.KH * p.KW >= 4 && (p.KW & 1) && !p.n_split && !p.res && !p.up2 && !p.res_up2 &&
           conv_span_max(p, SPAN_BM) <= SPAN_ROWS;
}

// VTF_DMA3_WIDE_TAIL=1 (read per launch): bf16x3 convs also split last rounds of more than half
// the slots.  One lane: the 840-tile convs 415 -> 390 us; four lanes (c3): -3.5 %, the other lanes'
// work already fills those slots and the slices add slab traffic (profiles/r06_dma3_wide_tail_ab.txt)
bool dma3_wide_tail() {
    const char* e = std::getenv("VTF_DMA3_WIDE_TAIL");
    return e && std::atoi(e) != 0;
}

template <int BM, int BN, int WGM>
void launch_dma3_t(ConvParams p, hipStream_t st) {
    p.gx = (int)cdiv(p.M, BM);
    p.gy = (int)cdiv(p.Cout, BN);
    p.group_m = dma_group_m();
    p.zero = zero_page(stream_device(st));
    const int T = p.gx * p.gy, KT = (p.K + 31) / 32;
    const int slots = 2 * cu_count();
    p.dp_tiles = T;
    p.tail_split = 1;
    p.split = 1;
    if (p.split_fp32 && !splitk_disabled()) {
        if (T > slots) {
            const int R = T % slots;
            const int S = R > 0 ? std::min(slots / R, KT / 4) : 0;
            if (R > 0 && R <= slots / 2 && S >= 2) {
                p.dp_tiles = T - R;
                p.tail_split = S;
            } else if (R > slots / 2 && dma3_wide_tail()) {
                // a last round of more than half the slots (YOLO's 13x13-scale 3x3 convs: 840 tiles
                // on 512 slots, the second round 64 % full): split those R tiles into S K-slices,
                // S chosen for the fewest tile-rounds ceil(R S / slots) / S (840: S = 3, 2 -> 1.67)
                int best = 1;
                double cost = 1.0;
                for (int s = 2; s <= 8 && KT / s >= 4; s++) {
                    const double c = (double)((R * s + slots - 1) / slots) / s;
                    if (c < cost - 1e-9) {
                        cost = c;
                        best = s;
                    }
                }
                if (best > 1 && cost <= 0.85) {
                    p.dp_tiles = T - R;
                    p.tail_split = best;
                }
            }
        } else {
            const int S = std::min(std::min(slots / T, KT / 4), 16);
            if (S >= 2) {
                p.dp_tiles = 0;
                p.tail_split = S;
            }
        }
    }
    const int nt = T - p.dp_tiles;
    p.ws = nt ? dma_ws(st, (size_t)nt * p.tail_split * BM * BN * 4) : nullptr;
    k_conv_dma3<BM, BN, WGM><<<(unsigned)(p.dp_tiles + nt * p.tail_split), 256, 0, st>>>(p);
    // the slab layout (wave, fragment, lane) is MODE 1's for the same tile / wave grid
    if (nt) k_conv_dma_tail<1, BM, BN, WGM, 2, 2><<<(unsigned)(nt * (BM / 16) * (BN > 64 ? BN / 64 : 1)), 256, 0, st>>>(p);
}

}  // namespace

// (vtf_release_stream, capi.hip)
void release_dma_ws(hipStream_t st) { release_dma_ws_impl(st); }


// conv (split pairs, bias + PReLU) + MaxPool2d(k, s, ceil_mode=True) in one launch
// (k_conv_span_pool); false (nothing launched) when the shape does not fit its tiles
constexpr int SPOOL_BM = 256, SPOOL_SPAN = 368;
bool launch_conv_span_pool(ConvParams p, int k, int s, void* pout, int& POH, int& POW, hipStream_t st) {
    const char* e = std::getenv("VTF_CONV_SPAN_POOL");
    if ((e && std::atoi(e) == 0) || !p.in_sp || p.s3 || p.sh != 1 || p.sw != 1 || p.ph || p.pw || p.Cin != 32 ||
        (p.in_cstride && p.in_cstride != p.Cin) || p.Cout > 64 || p.Cout % 8 || !(p.KW & 1) || p.res || p.up2 ||
        p.n_split || p.alpha || p.relu || p.leaky || p.gelu || p.scale != 1.f || p.out_sp || p.N <= 0)
        return false;
    auto pool_out = [](int L, int k_, int s_) {  // torch pooling_output_shape, padding 0, ceil_mode
        int o = ((L - k_ + s_ - 1) / s_) + 1;
        if ((o - 1) * s_ >= L) o--;
        return o;
    };
    SpanPool sp{};
    sp.k = k;
    sp.s = s;
    sp.POH = pool_out(p.OH, k, s);
    sp.POW = pool_out(p.OW, k, s);
    sp.out = pout;
    const int HW = p.H * p.W;
    if (p.OH * p.OW <= SPOOL_BM) {
        sp.parts = 1;
        sp.cg = SPOOL_BM / (p.OH * p.OW);
        sp.PH2 = sp.POH;
        sp.RP = p.OH;
    } else {
        sp.cg = 1;
        for (sp.parts = 2; sp.parts <= sp.POH; sp.parts++) {
            sp.PH2 = (sp.POH + sp.parts - 1) / sp.parts;
            sp.RP = std::min(p.OH, (sp.PH2 - 1) * s + k);
            if (sp.RP * p.OW <= SPOOL_BM) break;
        }
        if (sp.parts > sp.POH) return false;
    }
    const int span = (sp.cg - 1) * HW + (sp.RP + p.KH - 1) * p.W;
    if (span > SPOOL_SPAN || sp.cg * sp.RP * p.OW > SPOOL_BM) return false;
    p.zero = zero_page(stream_device(st));
    const int grid = sp.parts == 1 ? (int)cdiv(p.N, sp.cg) : p.N * sp.parts;
    // B stages (VTF_SPOOL_NS, experiments): 2 / 3 / 4 measured 288 / 292 / 295 us per launch on
    // c2 (the weight round trip is not what bounds it)
    static const int ns = [] {
        const char* e = std::getenv("VTF_SPOOL_NS");
        return e ? std::atoi(e) : 2;
    }();
    if (ns == 3)
        k_conv_span_pool<SPOOL_BM, 64, SPOOL_SPAN, 3><<<(unsigned)grid, 256, 0, st>>>(p, sp);
    else if (ns == 4)
        k_conv_span_pool<SPOOL_BM, 64, SPOOL_SPAN, 4><<<(unsigned)grid, 256, 0, st>>>(p, sp);
    else if (p.Cout <= 48)
        k_conv_span_pool<SPOOL_BM, 64, SPOOL_SPAN, 2, 3><<<(unsigned)grid, 256, 0, st>>>(p, sp);
    else
        k_conv_span_pool<SPOOL_BM, 64, SPOOL_SPAN, 2><<<(unsigned)grid, 256, 0, st>>>(p, sp);
    POH = sp.POH;
    POW = sp.POW;
    return true;
}

bool conv_dma_ok(const ConvParams& p) {
    // the 16-B pieces need 8-channel granules; the staged epilogue 8-channel groups
    return p.Cin % 8 == 0 && (p.in_cstride == 0 || p.in_cstride % 8 == 0) && p.Cout % 8 == 0 && p.out_cstride % 8 == 0 &&
           p.out_coff % 8 == 0 && (!p.res || p.res_cstride % 8 == 0) &&
           (!p.n_split || (p.n_split % 8 == 0 && p.out2_cstride % 8 == 0 && p.out2_coff % 8 == 0));
}

int conv_dma_choice_bf16(const ConvParams& p) {
    // per-layer A/B on FaceNet (batch 128, profiles/r02o_facenet_layers_*): k_conv's small
    // register-staged tiles win on 32-channel outputs and on K < 256 (1-4 k-steps); the 2-stage
    // 128 x 128 / 256 x 64 DMA tiles on grids of at least one whole round; the 3-stage 64 x 64 DMA
    // tiles on 1x1 and strided convs and on the 3x3-spatial Block8 maps (M <= 2048); k_conv keeps
    // the padded 1x7 / 7x1 / 3x3 convs of the small maps
    static const int force = [] {
        const char* e = std::getenv("VTF_DMA_BF16");  // -1 auto, 0 k_conv, 1 large tiles, 2 small tiles
        return e ? std::atoi(e) : -1;
    }();
    if (!conv_dma_ok(p)) return 0;
    if (force >= 0) return force;
    if (p.Cout <= 32 || p.K < 256) return 0;
    const int bm = p.Cout <= 64 ? 256 : 128, bn = p.Cout <= 64 ? 64 : 128;
    if (cdiv(p.M, bm) * cdiv(p.Cout, bn) >= 2 * cu_count()) return 1;
    if (p.KH * p.KW == 1 || p.M <= 2048 || p.sh > 1 || p.sw > 1) return 2;
    return 0;
}

void launch_conv_dma(const ConvParams& p, bool bf16, hipStream_t st) {
    if (p.M <= 0) return;
    VTF_CHECK(conv_dma_ok(p), VTF_E_ARG, "conv_dma: channel counts / strides must be multiples of 8");
    if (p.s3) {
        // bf16x3: 128 x 64 tiles up to 64 output channels, 64 x 128 above
        if (p.Cout <= 64)
            launch_dma3_t<128, 64, 2>(p, st);
        else
            launch_dma3_t<64, 128, 2>(p, st);
        return;
    }
    VTF_CHECK(bf16 || p.in_sp, VTF_E_ARG, "conv_dma: bf16 or split-pair operands");
    VTF_CHECK(!p.out_sp || !bf16, VTF_E_ARG, "conv_dma: split-pair output is an fp32-mode output");
    if (bf16) {
        // grids below a whole round of large tiles (FaceNet Block35 / 17 / 8): 64 x 64 tiles, three
        // stages (two k-steps in flight) at 3 workgroups per CU
        if (conv_dma_choice_bf16(p) == 2) {
            launch_dma_t<0, 64, 64, 2, 3, 3>(p, st);
            return;
        }
        // Cout an odd multiple of 64 (FaceNet's 192-channel convs): 256 x 64 tiles instead of 128 x
        // 128 ones whose last column block is half empty (FaceNet forward 1.790 -> 1.751 ms per 128
        // faces, profiles/r06_facenet_n64_ab.txt; VTF_DMA_N64=0: off)
        static const bool n64_on = [] {
            const char* e = std::getenv("VTF_DMA_N64");
            return !(e && std::atoi(e) == 0);
        }();
        const bool n64 = n64_on && p.Cout % 128 != 0 && p.Cout % 64 == 0;
        if (p.Cout <= 32)
            launch_dma_t<0, 256, 32, 4>(p, st);
        else if (p.Cout <= 64 || n64)
            launch_dma_t<0, 256, 64, 4>(p, st);
        else
            launch_dma_t<0, 128, 128, 2>(p, st);
    } else {
        // split mode, <= 64 channels (MTCNN RNet / ONet convs, K = 192..576: 6-18 k-steps, so the
        // per-tile prologue / epilogue latency weighs): 128 x 64 tiles at 3 workgroups per CU hide
        // more of it than 256 x 64 tiles at 2 (VTF_DMA_SPLIT64=256 for the latter)
        static const int big = [] {
            const char* e = std::getenv("VTF_DMA_SPLIT64");
            return e ? std::atoi(e) : 128;
        }();
        if (conv_span_ok(p)) {
            if (p.Cin == 32)
                launch_span_t<1, SPAN_BM, 64, 2, SPAN_ROWS, 3, 2>(p, st);
            else
                launch_span_t<2, SPAN_BM, 64, 2, SPAN_ROWS, 2, 2>(p, st);
            return;
        }
        if (p.Cout <= 64 && big == 256)
            launch_dma_t<1, 256, 64, 4>(p, st);
        else if (p.Cout <= 64 && big == 64)
            launch_dma_t<1, 64, 64, 2, 3, 3>(p, st);
        else if (p.Cout <= 64 && big == 129)
            launch_dma_t<1, 128, 64, 2, 2, 3>(p, st);
        else if (p.Cout <= 64)
            launch_dma_t<1, 128, 64, 2, 3>(p, st);
        else
            launch_dma_t<1, 128, 128, 2>(p, st);
    }
}

}  // namespace vtf

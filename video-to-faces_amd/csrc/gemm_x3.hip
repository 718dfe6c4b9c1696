// fp32-grade GEMM on the fp16 matrix cores with pre-split operands (gfx950).
//
// Replaces the nn.Linear layers of the ViT blocks (src/videotofaces/encoders/vit.py:29-37:
// q|k|v, proj, fc1, fc2) in the split-fp16 mode.  k_conv's split mode (conv.hip) split every
// fp32 operand element at LDS staging: per 32-deep step each thread loaded fp32 vectors into
// registers, converted them to two fp16 planes with VALU and stored them with ds_write_b64 --
// the staging (load latency, split VALU, LDS writes) bounded it at ~0.18 of the split peak.
// Here the operands arrive split ("SP" layout, gemm_x3.hpp): the producers (LayerNorm, attention,
// the fc1 epilogue) write x0/x1 once, the weights are split once on the host, and the tiles
// go HBM -> LDS by LDS-DMA (global_load_lds_dwordx4): no staging VGPRs, no staging VALU.
//
// Tile 128 x 128 per 256-thread workgroup (2 x 2 waves of 64 x 64 = 4 x 4 fragments), 32-deep
// k-steps, two LDS stages (64 KB; two workgroups per CU): the DMA of step k+1 is in flight while
// step k runs on the MFMA; one barrier per step.  Per step and fragment pair three
// v_mfma_f32_16x16x32_f16: x0 w0 into acc, x0 w1 + x1 w0 into accx (the same chains and order
// as k_conv's split mode, so the results are bit-identical to it), combined once at the end.
//
// LDS image of a stage: rows of 128 B (the 32-deep k-step of one row: 4 chunks x 2 planes of
// 16 B), 16-B slot s of row r holds (plane, chunk) = s ^ ((r >> 1) & 7) split as (s' >> 2, s' & 3).
// One DMA wave-instruction writes 1 KB = 8 whole rows lane-linearly, so the swizzle is applied
// on the global source address; the fragment reads (ds_read_b128, rows lane & 15, chunk
// lane >> 4) then hit 16 distinct slots per 16-lane bank group: conflict-free.
#include <algorithm>
#include <cstdlib>
#include <cmath>
#include <cstring>
#include <map>
#include <mutex>
#include <vector>

#include "common.hpp"
#include "gemm_x3.hpp"

namespace vtf {

namespace {

typedef __attribute__((ext_vector_type(8))) _Float16 h8;
typedef __attribute__((ext_vector_type(4))) float f4;

// fused epilogue of one tile from its fp32 LDS image E [BM][BN + 4]: each thread finishes 8
// consecutive channels of a row (bias, residual, GELU; fp32 or SP stores, 16-byte accesses)
template <int BM, int BN, int NT = 256>
__device__ inline void tile_epilogue(const GemmX3Params& p, const float* E, int64_t m0, int n0) {
    constexpr int LDE = BN + 4;
    const int tid = threadIdx.x, lane = tid & 63;
    constexpr int G = BN / 8;
    static_assert(NT % G == 0, "epilogue groups");
    const int g = tid % G, c0 = n0 + 8 * g;
    if (c0 >= p.N) return;
    float b8[8];
#pragma unroll
    for (int e = 0; e < 8; e++) b8[e] = p.bias ? p.bias[c0 + e] : 0.f;
    bool bad = false;
    for (int r = tid / G; r < BM; r += NT / G) {
        const int64_t m = m0 + r;
        if (m >= p.M) break;
        const f4 lo = *(const f4*)(E + r * LDE + 8 * g), hi = *(const f4*)(E + r * LDE + 8 * g + 4);
        float v[8] = {lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]};
        float rv[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if (p.res) {
            const f4 r0 = *(const f4*)(p.res + m * p.ldr + c0), r1 = *(const f4*)(p.res + m * p.ldr + c0 + 4);
            rv[0] = r0[0], rv[1] = r0[1], rv[2] = r0[2], rv[3] = r0[3];
            rv[4] = r1[0], rv[5] = r1[1], rv[6] = r1[2], rv[7] = r1[3];
        }
#pragma unroll
        for (int e = 0; e < 8; e++) {
            float x = v[e];
            if (p.bias) x = x + b8[e];
            if (p.res) x = x + rv[e];
            if (p.gelu) x = 0.5f * x * (1.0f + erff(x * 0.70710678118654752f));
            v[e] = x;
        }
        if (p.out_sp) {
            char* row = (char*)p.out + m * (int64_t)p.N * 4;
            sp_store4(row, c0, v[0], v[1], v[2], v[3], bad);
            sp_store4(row, c0 + 4, v[4], v[5], v[6], v[7], bad);
        } else {
            float* o = (float*)p.out + m * p.ldo + c0;
            *(f4*)o = f4{v[0], v[1], v[2], v[3]};
            *(f4*)(o + 4) = f4{v[4], v[5], v[6], v[7]};
        }
    }
    if (p.ovf && __ballot(bad) && lane == 0) atomicOr(p.ovf, 1);
}

// NW waves as (NW / 2) x 2, each a 64 x 64 output block (4 x 4 fragments); the epilogue stages
// 128 rows at a time through the stage memory
template <int BM, int BN, int NW>
__global__ __launch_bounds__(64 * NW, 8 / NW) void k_gemm_x3(GemmX3Params p) {
    constexpr int NT = 64 * NW;
    constexpr int RB = 128;  // LDS bytes per row and k-step
    constexpr int A_ST = BM * RB, ST = (BM + BN) * RB;
    constexpr int LDE = BN + 4;
    constexpr int ER = 128;  // epilogue rows per pass
    constexpr int SM = 2 * ST > ER * LDE * 4 ? 2 * ST : ER * LDE * 4;
    constexpr int WM = BM / (NW / 2), WN = BN / 2, FM = WM / 16, FN = WN / 16;
    constexpr int PA = BM / (8 * NW), PB = BN / (8 * NW);  // 1-KB DMA pieces per wave and stage
    static_assert(BM % (8 * NW) == 0 && BN % (8 * NW) == 0 && WM == 64 && WN == 64 && BM % ER == 0, "tile");
    __shared__ __attribute__((aligned(16))) char smem[SM];

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wm = wave >> 1, wn = wave & 1;
    // Work item: blockIdx.x < dp_tiles = one whole tile (data-parallel rounds); the rest are the
    // tail tiles' K slices (split-K over tail_split slices, reduced in-launch by the last
    // arriving slice).  Whole tiles are dealt XCD-aware: every XCD owns one contiguous run of
    // tile ids (workgroups go to XCDs round-robin by id); tile ids walk groups of group_m
    // M-tiles x all N-tiles, so the A row-blocks and B column-blocks an XCD's resident
    // workgroups share stay in its L2.  (Placement only affects speed; any bijection is correct.)
    const int bid = blockIdx.x;
    const bool tail = bid >= p.dp_tiles;
    int t, slice = 0;
    if (!tail) {
        const int xcd = bid & 7, loc = bid >> 3, per = p.dp_tiles >> 3, rem = p.dp_tiles & 7;
        t = xcd < rem ? xcd * (per + 1) + loc : rem * (per + 1) + (xcd - rem) * per + loc;
    } else {
        t = p.dp_tiles + (bid - p.dp_tiles) / p.tail_split;
        slice = (bid - p.dp_tiles) % p.tail_split;
    }
    const int gm = p.group_m > 0 ? p.group_m : p.gx;
    const int span = gm * p.gy, first = (t / span) * gm, gsz = min(p.gx - first, gm);
    const int tile_m = first + (t % span) % gsz, tile_n = (t % span) / gsz;
    const int64_t m0 = (int64_t)tile_m * BM;
    const int n0 = tile_n * BN;

    // DMA sources: piece j of this wave = rows 8 (wave + NW j) .. +7; the lane's LDS slot lane & 7
    // of row 8 (wave + NW j) + (lane >> 3) takes source slot (lane & 7) ^ h, h = (row >> 1) & 7
    const int src = (lane & 7) ^ (((lane >> 4) + 4 * (wave & 1)) & 7);
    const int soff = (src & 3) * 32 + (src >> 2) * 16;
    const int64_t rowa = p.lda, rowb = p.ldb;
    const char* ga[PA];
    const char* gb[PB];
#pragma unroll
    for (int j = 0; j < PA; j++) {
        const int64_t m = min(m0 + 8 * (wave + NW * j) + (lane >> 3), p.M - 1);
        ga[j] = (const char*)p.a + m * rowa + soff;
    }
#pragma unroll
    for (int j = 0; j < PB; j++) {
        const int64_t n = min(n0 + 8 * (wave + NW * j) + (lane >> 3), p.N - 1);
        gb[j] = (const char*)p.b + n * rowb + soff;
    }
    auto issue = [&](int kt, int s) {
        const int64_t kb = (int64_t)kt * RB;
        char* base = smem + s * ST;
#pragma unroll
        for (int j = 0; j < PA; j++)
            __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(ga[j] + kb),
                                             (void __attribute__((address_space(3)))*)(base + (wave + NW * j) * 1024), 16,
                                             0, 0);
#pragma unroll
        for (int j = 0; j < PB; j++)
            __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(gb[j] + kb),
                                             (void __attribute__((address_space(3)))*)(base + A_ST + (wave + NW * j) * 1024),
                                             16, 0, 0);
    };

    f4 acc[FM][FN], accx[FM][FN];
#pragma unroll
    for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) {
            acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
            accx[i][j] = f4{0.f, 0.f, 0.f, 0.f};
        }
    // fragment read offsets: row (lane & 15) of a 16-row block, chunk lane >> 4, plane pl
    const int hsw = (lane & 15) >> 1;
    const int o0 = (lane & 15) * RB + (((lane >> 4) ^ hsw) << 4);      // plane 0
    const int o1 = (lane & 15) * RB + (((4 + (lane >> 4)) ^ hsw) << 4);  // plane 1

    const int KT = p.K / 32;
    const int kt0 = tail ? (int)((int64_t)slice * KT / p.tail_split) : 0;
    const int kt1 = tail ? (int)((int64_t)(slice + 1) * KT / p.tail_split) : KT;
    issue(kt0, 0);
    for (int kt = kt0; kt < kt1; kt++) {
        // this wave's pieces of step kt have landed; after the barrier every wave's have, and
        // every wave is done reading the other stage (its MFMAs consumed those reads)
        asm volatile("s_waitcnt vmcnt(0)\n\ts_barrier" ::: "memory");
        const int sb = (kt - kt0) & 1;
        if (kt + 1 < kt1) issue(kt + 1, sb ^ 1);
        const char* As = smem + sb * ST + wm * WM * RB;
        const char* Bs = smem + sb * ST + A_ST + wn * WN * RB;
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
    }
    __syncthreads();  // no DMA outstanding; every wave is done with the stages
    if (tail) {
        // K slice of a tail tile: the fp32 partial (fragment order: 16-B stores, coalesced) to the
        // workspace; k_gemm_x3_tail sums the slices in order and runs the epilogue.  (An in-launch
        // last-arriver reduction needs agent-scope release/acquire fences, which write back and
        // invalidate the XCD's L2 under the whole-tile workgroups still streaming from it:
        // measured 20% slower on ViT-L.)
        f4* slab = (f4*)(p.ws + ((int64_t)(t - p.dp_tiles) * p.tail_split + slice) * (BM * BN));
#pragma unroll
        for (int i = 0; i < FM; i++)
#pragma unroll
            for (int j = 0; j < FN; j++) slab[((wave * FM + i) * FN + j) * 64 + lane] = acc[i][j] + accx[i][j] * 0.00048828125f;
        return;
    }
    float* E = (float*)smem;
#pragma unroll
    for (int ph = 0; ph < BM / ER; ph++) {
        if (ph) __syncthreads();  // the previous pass's rows are finished
        if (wm * WM / ER == ph) {
#pragma unroll
            for (int j = 0; j < FN; j++)
#pragma unroll
                for (int i = 0; i < FM; i++) {
                    const f4 v = acc[i][j] + accx[i][j] * 0.00048828125f;
#pragma unroll
                    for (int q = 0; q < 4; q++)
                        E[(wm * WM - ph * ER + i * 16 + 4 * (lane >> 4) + q) * LDE + wn * WN + j * 16 + (lane & 15)] = v[q];
                }
        }
        __syncthreads();
        tile_epilogue<ER, BN, NT>(p, E, m0 + ph * ER, n0);
    }
}

// Ping-pong variant: 256 x 128 tiles, 8 waves in two groups of four by M half (group g = wave >> 2
// holds rows 128 g .. +127 as 2 x 2 waves of 64 x 64; waves w and w + 4 share a SIMD), three LDS
// stages (144 KB, one workgroup per CU).  A k-step is two phases per wave -- fragment reads, then
// 24 MFMAs -- each closed by a workgroup barrier, and group 1 runs one barrier behind group 0: at
// every barrier the groups swap roles, so each SIMD's matrix pipe alternates between its two
// waves while the other one reads LDS.  The DMA of step k + 2 is issued in the second read phase
// of step k and waited for with a counted vmcnt before the barrier that precedes every read of it
// (group 0 after its second MFMA phase, group 1 after its second read phase: the same barrier).
// Same LDS image, MFMA chains and order per output as k_gemm_x3 (bit-identical results); the
// tail split and slab layout are k_gemm_x3<256, 128, 8>'s.
__device__ inline void pp_barrier() { asm volatile("s_barrier" ::: "memory"); }

__global__ __launch_bounds__(512, 1) void k_gemm_x3_pp(GemmX3Params p) {
    constexpr int BM = 256, BN = 128, NW = 8, NT = 512, NS = 3;
    constexpr int RB = 128, A_ST = BM * RB, ST = (BM + BN) * RB, LDE = BN + 4, ER = 128;
    constexpr int SM = NS * ST;
    constexpr int FN = 4, PA = BM / (8 * NW), PB = BN / (8 * NW), P = PA + PB;
    static_assert(SM <= 160 * 1024 && ER * LDE * 4 <= SM && P == 6, "ping-pong tile");
    __shared__ __attribute__((aligned(16))) char smem[SM];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int grp = wave >> 2, wmg = wave >> 1, wn = wave & 1;  // wmg: 64-row block 0..3
    const int bid = blockIdx.x;
    const bool tail = bid >= p.dp_tiles;
    int t, slice = 0;
    if (!tail) {
        const int xcd = bid & 7, loc = bid >> 3, per = p.dp_tiles >> 3, rem = p.dp_tiles & 7;
        t = xcd < rem ? xcd * (per + 1) + loc : rem * (per + 1) + (xcd - rem) * per + loc;
    } else {
        t = p.dp_tiles + (bid - p.dp_tiles) / p.tail_split;
        slice = (bid - p.dp_tiles) % p.tail_split;
    }
    const int gm = p.group_m > 0 ? p.group_m : p.gx;
    const int span = gm * p.gy, first = (t / span) * gm, gsz = min(p.gx - first, gm);
    const int tile_m = first + (t % span) % gsz, tile_n = (t % span) / gsz;
    const int64_t m0 = (int64_t)tile_m * BM;
    const int n0 = tile_n * BN;
    const int src = (lane & 7) ^ (((lane >> 4) + 4 * (wave & 1)) & 7);
    const int soff = (src & 3) * 32 + (src >> 2) * 16;
    const int64_t rowa = p.lda, rowb = p.ldb;
    const char* ga[PA];
    const char* gb[PB];
#pragma unroll
    for (int j = 0; j < PA; j++) {
        const int64_t m = min(m0 + 8 * (wave + NW * j) + (lane >> 3), p.M - 1);
        ga[j] = (const char*)p.a + m * rowa + soff;
    }
#pragma unroll
    for (int j = 0; j < PB; j++) {
        const int64_t n = min(n0 + 8 * (wave + NW * j) + (lane >> 3), p.N - 1);
        gb[j] = (const char*)p.b + n * rowb + soff;
    }
    auto issue = [&](int kt, int s) {
        const int64_t kb = (int64_t)kt * RB;
        char* base = smem + s * ST;
#pragma unroll
        for (int j = 0; j < PA; j++)
            __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(ga[j] + kb),
                                             (void __attribute__((address_space(3)))*)(base + (wave + NW * j) * 1024), 16,
                                             0, 0);
#pragma unroll
        for (int j = 0; j < PB; j++)
            __builtin_amdgcn_global_load_lds((const void __attribute__((address_space(1)))*)(gb[j] + kb),
                                             (void __attribute__((address_space(3)))*)(base + A_ST + (wave + NW * j) * 1024),
                                             16, 0, 0);
    };
    // wait until at most `newer` later steps' DMA pieces of this wave are outstanding
    auto wait_dma = [&](int newer) {
        if (newer > 0)
            asm volatile("s_waitcnt vmcnt(%0)" ::"n"(P) : "memory");
        else
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    };
    f4 acc[4][FN], accx[4][FN];
#pragma unroll
    for (int i = 0; i < 4; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) {
            acc[i][j] = f4{0.f, 0.f, 0.f, 0.f};
            accx[i][j] = f4{0.f, 0.f, 0.f, 0.f};
        }
    const int hsw = (lane & 15) >> 1;
    const int o0 = (lane & 15) * RB + (((lane >> 4) ^ hsw) << 4);
    const int o1 = (lane & 15) * RB + (((4 + (lane >> 4)) ^ hsw) << 4);
    const int KT = p.K / 32;
    const int kt0 = tail ? (int)((int64_t)slice * KT / p.tail_split) : 0;
    const int kt1 = tail ? (int)((int64_t)(slice + 1) * KT / p.tail_split) : KT;
    issue(kt0, 0);
    if (kt0 + 1 < kt1) issue(kt0 + 1, 1);
    wait_dma(kt0 + 1 < kt1 ? 1 : 0);
    pp_barrier();  // step kt0 visible to every wave
    if (grp) pp_barrier();  // the stagger: group 1 one barrier behind
    for (int kt = kt0; kt < kt1; kt++) {
        const int sb = (kt - kt0) % NS;
        const char* As = smem + sb * ST + wmg * 64 * RB;
        const char* Bs = smem + sb * ST + A_ST + wn * 64 * RB;
        h8 b0[FN], b1[FN], a0[2], a1[2];
        // ---- phase 1: B and A rows 0, 1 -> 24 MFMAs
#pragma unroll
        for (int j = 0; j < FN; j++) {
            b0[j] = *(const h8*)(Bs + j * 16 * RB + o0);
            b1[j] = *(const h8*)(Bs + j * 16 * RB + o1);
        }
#pragma unroll
        for (int i = 0; i < 2; i++) {
            a0[i] = *(const h8*)(As + i * 16 * RB + o0);
            a1[i] = *(const h8*)(As + i * 16 * RB + o1);
        }
        pp_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int j = 0; j < FN; j++) {
                acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0[i], b0[j], acc[i][j], 0, 0, 0);
                accx[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0[i], b1[j], accx[i][j], 0, 0, 0);
                accx[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[i], b0[j], accx[i][j], 0, 0, 0);
            }
        __builtin_amdgcn_s_setprio(0);
        pp_barrier();
        // ---- phase 2: the DMA of step kt + 2 (its stage was last read in step kt - 1, by every
        //      wave before the barrier that opened this step's first MFMA phase... of group 1), A
        //      rows 2, 3 -> 24 MFMAs
        if (kt + 2 < kt1) issue(kt + 2, (kt - kt0 + 2) % NS);
#pragma unroll
        for (int i = 0; i < 2; i++) {
            a0[i] = *(const h8*)(As + (i + 2) * 16 * RB + o0);
            a1[i] = *(const h8*)(As + (i + 2) * 16 * RB + o1);
        }
        if (grp && kt + 1 < kt1) wait_dma(kt + 2 < kt1 ? 1 : 0);  // step kt + 1 (group 1)
        pp_barrier();
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int i = 0; i < 2; i++)
#pragma unroll
            for (int j = 0; j < FN; j++) {
                acc[i + 2][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0[i], b0[j], acc[i + 2][j], 0, 0, 0);
                accx[i + 2][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0[i], b1[j], accx[i + 2][j], 0, 0, 0);
                accx[i + 2][j] = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1[i], b0[j], accx[i + 2][j], 0, 0, 0);
            }
        __builtin_amdgcn_s_setprio(0);
        if (!grp && kt + 1 < kt1) wait_dma(kt + 2 < kt1 ? 1 : 0);  // step kt + 1 (group 0)
        pp_barrier();
    }
    if (!grp) pp_barrier();  // (group 1's extra barrier at the start)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();  // no DMA outstanding; every wave is done with the stages
    if (tail) {
        f4* slab = (f4*)(p.ws + ((int64_t)(t - p.dp_tiles) * p.tail_split + slice) * (BM * BN));
#pragma unroll
        for (int i = 0; i < 4; i++)
#pragma unroll
            for (int j = 0; j < FN; j++) slab[((wave * 4 + i) * FN + j) * 64 + lane] = acc[i][j] + accx[i][j] * 0.00048828125f;
        return;
    }
    float* E = (float*)smem;
#pragma unroll
    for (int ph = 0; ph < BM / ER; ph++) {
        if (ph) __syncthreads();
        if (wmg * 64 / ER == ph) {
#pragma unroll
            for (int j = 0; j < FN; j++)
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const f4 v = acc[i][j] + accx[i][j] * 0.00048828125f;
#pragma unroll
                    for (int q = 0; q < 4; q++)
                        E[(wmg * 64 - ph * ER + i * 16 + 4 * (lane >> 4) + q) * LDE + wn * 64 + j * 16 + (lane & 15)] = v[q];
                }
        }
        __syncthreads();
        tile_epilogue<ER, BN, NT>(p, E, m0 + ph * ER, n0);
    }
}

// tail tiles: 2 x BM / 16 workgroups per tile, each sums the K slices of one 16-row x 64-column
// block (the 4 fragments with that wm, i, wn: one f4 per thread) in slice order (deterministic)
// into an LDS image of the block, then the shared epilogue over those 16 rows x 64 columns
template <int BM, int BN, int NW>
__global__ __launch_bounds__(256) void k_gemm_x3_tail(GemmX3Params p) {
    constexpr int WN = BN / 2, LDE = WN + 4, WM = 64, FM = WM / 16, FN = WN / 16, NB = 2 * BM / 16;
    static_assert(BN == 128, "tail reduce layout: 16-row blocks of 2 waves x 4 fragments");
    __shared__ __attribute__((aligned(16))) float E[16 * LDE];
    const int tid = threadIdx.x;
    const int tt = blockIdx.x / NB, part = blockIdx.x % NB, wn = part & 1, wm = (part >> 1) / FM, i = (part >> 1) % FM;
    const int t = p.dp_tiles + tt;
    const int gm = p.group_m > 0 ? p.group_m : p.gx;
    const int span = gm * p.gy, first = (t / span) * gm, gsz = min(p.gx - first, gm);
    const int tile_m = first + (t % span) % gsz, tile_n = (t % span) / gsz;
    const f4* s0 = (const f4*)(p.ws + (int64_t)tt * p.tail_split * (BM * BN));
    {
        const int j = tid >> 6, lane = tid & 63;  // 256 f4: j (2 bits) | lane (6 bits)
        const int idx = (((2 * wm + wn) * FM + i) * FN + j) * 64 + lane;
        f4 v = s0[idx];
        for (int z = 1; z < p.tail_split; z++) v = v + s0[(int64_t)z * (BM * BN / 4) + idx];
#pragma unroll
        for (int q = 0; q < 4; q++) E[(4 * (lane >> 4) + q) * LDE + j * 16 + (lane & 15)] = v[q];
    }
    __syncthreads();
    tile_epilogue<16, WN>(p, E, (int64_t)tile_m * BM + wm * WM + i * 16, tile_n * BN + wn * WN);
}

// one thread per 8-element chunk
__global__ void k_split_rows(const float* __restrict__ x, int64_t rows, int K, int64_t ld, char* __restrict__ out,
                             int* __restrict__ ovf) {
    const int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    const int KC = K / 8;
    bool bad = false;
    if (i < rows * KC) {
        const int64_t r = i / KC;
        const int c = (int)(i % KC);
        const f4 lo = *(const f4*)(x + r * ld + 8 * c), hi = *(const f4*)(x + r * ld + 8 * c + 4);
        char* row = out + r * (int64_t)K * 4;
        sp_store4(row, 8 * c, lo[0], lo[1], lo[2], lo[3], bad);
        sp_store4(row, 8 * c + 4, hi[0], hi[1], hi[2], hi[3], bad);
    }
    if (ovf && __ballot(bad) && (threadIdx.x & 63) == 0) atomicOr(ovf, 1);
}

int gemm_group_m() {
    static int g = [] {
        const char* e = std::getenv("VTF_CONV_GROUP_M");
        return e ? std::atoi(e) : 8;
    }();
    return g;
}

// tail split-K (VTF_GEMM_TAIL=0 disables: every tile whole)
bool gemm_tail_on() {
    static bool on = [] {
        const char* e = std::getenv("VTF_GEMM_TAIL");
        return !(e && std::atoi(e) == 0);
    }();
    return on;
}

// per-(device, stream) tail workspace (fp32 slabs): grows x1.5; an outgrown buffer is retired,
// not freed (hipFree synchronises the device while other lanes' kernels may still use it)
float* tail_ws(hipStream_t st, size_t bytes) {
    static std::mutex mu;
    static std::map<std::pair<int, hipStream_t>, std::pair<float*, size_t>> m;
    static std::vector<void*> retired;
    std::lock_guard<std::mutex> g(mu);
    auto& w = m[{stream_device(st), st}];
    if (w.second < bytes) {
        if (w.first) retired.push_back(w.first);
        w.first = nullptr;
        w.second = 0;
        const size_t b = bytes + bytes / 2;
        VTF_HIP(hipMalloc((void**)&w.first, b));
        w.second = b;
    }
    return w.first;
}

int device_cu_count() {
    static int cus = [] {
        int dev = 0, n = 256;
        if (hipGetDevice(&dev) == hipSuccess) (void)hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev);
        return n;
    }();
    return cus;
}

}  // namespace

template <int BM, int BN, int NW>
void launch_t(GemmX3Params p, hipStream_t st);
void launch_pp(GemmX3Params p, hipStream_t st);

// 256 x 128 tiles of 8 waves for large M: a third less operand traffic per FLOP than 128 x 128,
// but one workgroup per CU whose 8 waves share every barrier -- measured slower on ViT-L c4
// (6.3-6.5k vs 6.8k faces/s, profiles/r02o_*), so opt-in (VTF_GEMM_BIG=1)
// VTF_GEMM_BIG: 1 = 256 x 128 / 8 waves / 2 stages; 5 = the ping-pong kernel (k_gemm_x3_pp); 0 =
// 128 x 128 / 4 waves / 2 stages at two workgroups per CU.  c4 on one box (scripts/r05_gemm.sh):
// 0: 7.12-7.39k, ping-pong 7.24k, 256 x 128 / 3 stages 6.77-6.78k, 128 x 128 at one workgroup
// per CU with 3 / 4 stages 5.78-5.79k / 5.72-5.76k faces/s (profiles/r05_gemm_variants_ab.txt)
static int big_tiles() {
    static int v = [] {
        const char* e = std::getenv("VTF_GEMM_BIG");
        return e ? std::atoi(e) : 0;
    }();
    return v;
}

void launch_gemm_x3(const GemmX3Params& p0, hipStream_t st) {
    if (p0.M <= 0) return;
    VTF_CHECK(p0.K > 0 && p0.K % 32 == 0 && p0.N > 0 && p0.N % 8 == 0, VTF_E_ARG, "gemm_x3: K % 32, N % 8");
    VTF_CHECK(p0.out_sp || p0.ldo >= p0.N, VTF_E_ARG, "gemm_x3: output stride");
    VTF_CHECK(!p0.res || (p0.ldr >= p0.N && p0.ldr % 4 == 0), VTF_E_ARG, "gemm_x3: residual stride");
    GemmX3Params p = p0;
    p.group_m = gemm_group_m();
    if (p.lda == 0) p.lda = (int64_t)p.K * 4;
    if (p.ldb == 0) p.ldb = (int64_t)p.K * 4;
    VTF_CHECK(p.lda >= (int64_t)p.K * 4 && p.ldb >= (int64_t)p.K * 4 && p.lda % 16 == 0 && p.ldb % 16 == 0, VTF_E_ARG,
              "gemm_x3: operand row strides");
    const int big = p.M >= 4096 ? big_tiles() : 0;
    if (big == 1) launch_t<256, 128, 8>(p, st);
    else if (big == 5) launch_pp(p, st);
    else launch_t<128, 128, 4>(p, st);
}

template <int BM, int BN, int NW>
void launch_t(GemmX3Params p, hipStream_t st) {
    p.gx = (int)cdiv(p.M, BM);
    p.gy = (int)cdiv(p.N, BN);
    const int T = p.gx * p.gy, KT = p.K / 32;
    // Rounds of whole tiles fill the chip's 2 x CUs workgroup slots; a last round holding only a
    // few tiles (M = 8320 token rows x N = 1024: 520 tiles on 512 slots) would run them on an
    // otherwise idle chip, so those tiles are split along K instead (>= 4 k-steps per slice)
    // and spread over the free slots.
    const int slots = (8 / NW) * device_cu_count();
    p.dp_tiles = T;
    p.tail_split = 1;
    if (gemm_tail_on() && T > slots) {
        const int R = T % slots;
        const int S = R > 0 ? std::min(slots / R, KT / 4) : 0;
        if (R > 0 && R <= slots / 2 && S >= 2) {
            p.dp_tiles = T - R;
            p.tail_split = S;
            p.ws = tail_ws(st, (size_t)R * S * BM * BN * 4);
        }
    }
    const int64_t grid = (int64_t)p.dp_tiles + (int64_t)(T - p.dp_tiles) * p.tail_split;
    k_gemm_x3<BM, BN, NW><<<(unsigned)grid, 64 * NW, 0, st>>>(p);
    if (p.dp_tiles < T) k_gemm_x3_tail<BM, BN, NW><<<(unsigned)(T - p.dp_tiles) * (2 * BM / 16), 256, 0, st>>>(p);
}

// the ping-pong kernel on the tile / tail plan of the 256 x 128 tiles at one workgroup per CU
void launch_pp(GemmX3Params p, hipStream_t st) {
    constexpr int BM = 256, BN = 128;
    p.gx = (int)cdiv(p.M, BM);
    p.gy = (int)cdiv(p.N, BN);
    const int T = p.gx * p.gy, KT = p.K / 32;
    const int slots = device_cu_count();
    p.dp_tiles = T;
    p.tail_split = 1;
    if (gemm_tail_on() && T > slots) {
        const int R = T % slots;
        const int S = R > 0 ? std::min(slots / R, KT / 4) : 0;
        if (R > 0 && R <= slots / 2 && S >= 2) {
            p.dp_tiles = T - R;
            p.tail_split = S;
            p.ws = tail_ws(st, (size_t)R * S * BM * BN * 4);
        }
    }
    const int64_t grid = (int64_t)p.dp_tiles + (int64_t)(T - p.dp_tiles) * p.tail_split;
    k_gemm_x3_pp<<<(unsigned)grid, 512, 0, st>>>(p);
    if (p.dp_tiles < T) k_gemm_x3_tail<BM, BN, 8><<<(unsigned)(T - p.dp_tiles) * (2 * BM / 16), 256, 0, st>>>(p);
}

void launch_split_rows(const float* x, int64_t rows, int K, int64_t ld, void* out, int* ovf, hipStream_t st) {
    const int64_t n = rows * (K / 8);
    if (n <= 0) return;
    k_split_rows<<<(unsigned)cdiv(n, 256), 256, 0, st>>>(x, rows, K, ld, (char*)out, ovf);
}

bool split_rows_host(const float* x, int64_t rows, int K, uint16_t* out) {
    bool ok = true;
    for (int64_t r = 0; r < rows; r++)
        for (int k = 0; k < K; k++) {
            const float v = x[r * K + k];
            ok &= std::fabs(v) < 16384.f;
            const _Float16 h0 = (_Float16)v;
            const _Float16 h1 = (_Float16)((v - (float)h0) * 2048.f);
            uint16_t* c = out + r * (int64_t)K * 2 + (k >> 3) * 16;
            std::memcpy(c + (k & 7), &h0, 2);
            std::memcpy(c + 8 + (k & 7), &h1, 2);
        }
    return ok;
}

}  // namespace vtf

using namespace vtf;

extern "C" int vtf_gemm_split(const float* d_a, const float* d_b, int64_t M, int N, int K, const float* d_bias,
                              float* d_out, void* hip_stream) {
    return guarded_on(stream_device((hipStream_t)hip_stream), [&] {
        VTF_CHECK(M >= 0 && N > 0 && K > 0 && K % 32 == 0 && N % 8 == 0, VTF_E_ARG,
                  "gemm_split: K % 32 == 0, N % 8 == 0");
        if (M == 0) return;
        VTF_CHECK(d_a && d_b && d_out, VTF_E_ARG, "null argument");
        hipStream_t st = (hipStream_t)hip_stream;
        char *sa = nullptr, *sb = nullptr;
        int* ovf = nullptr;
        VTF_HIP(hipMallocAsync((void**)&sa, (size_t)M * K * 4, st));
        VTF_HIP(hipMallocAsync((void**)&sb, (size_t)N * K * 4, st));
        VTF_HIP(hipMallocAsync((void**)&ovf, 4, st));
        VTF_HIP(hipMemsetAsync(ovf, 0, 4, st));
        launch_split_rows(d_a, M, K, K, sa, ovf, st);
        launch_split_rows(d_b, N, K, K, sb, ovf, st);
        GemmX3Params p{};
        p.a = sa;
        p.b = sb;
        p.out = d_out;
        p.bias = d_bias;
        p.M = M;
        p.N = N;
        p.K = K;
        p.ldo = N;
        launch_gemm_x3(p, st);
        int h_ovf = 0;
        VTF_HIP(hipMemcpyAsync(&h_ovf, ovf, 4, hipMemcpyDeviceToHost, st));
        VTF_HIP(hipFreeAsync(sa, st));
        VTF_HIP(hipFreeAsync(sb, st));
        VTF_HIP(hipFreeAsync(ovf, st));
        VTF_HIP(hipStreamSynchronize(st));
        VTF_CHECK(!h_ovf, VTF_E_ARG, "gemm_split: an operand is outside the fp16 range (|x| >= 2^14 or NaN)");
        VTF_HIP(hipGetLastError());
    });
}

// Fused front half of the MTCNN candidate nets (RNet stage 2 / ONet stage 3), one persistent
// workgroup per CU slot walking the candidates:
//
//   _get_cropped_candidates (mtcnn.py:153-163): the box crop adaptive-pooled to S x S from the
//     frame's summed-area table (exact integer bin sums, bit-exact bins);
//   conv1 (3 -> 28/32, 3x3) + PReLU + MaxPool2d(3, 2, ceil_mode=True)   (mtcnn.py:45-48, 83-86)
//   conv2 (28/32 -> 48/64, 3x3) + PReLU + MaxPool2d(3, 2, ceil_mode=True) (mtcnn.py:49-52, 87-90)
//
// Everything between the frame and the pool2 map stays in LDS; only the pool2 map
// ([n, 4, 4, 48] RNet / [n, 10, 10, 64] ONet, fp32 NHWC) reaches HBM, where the small remaining
// layers (conv3/conv4, the dense layer and the heads) run batched over all candidates.  The
// layer-by-layer path wrote and re-read the 23x23x32 pooled conv1 map (67.7 KB per ONet
// candidate) and the 21x21x64 conv2 map, and re-split every conv2 input element for each of
// its 9 taps.
//
// Both convs run on the fp16 matrix cores with split operands (x = x0 + x1 * 2^-11, three
// v_mfma_f32_16x16x32_f16 per 32-deep step: fp32-grade products, as the split-fp16 conv mode):
//   * the crop is stored split once, as planes [2][S+2][S+2][4] (channel 3 and the pad zero),
//     so conv1's k = ky*16 + kx*4 + c reads 8 contiguous halves per lane (2 k-steps of 32);
//   * pooled conv1 values are split once on their way into LDS, planes [2][P1*P1][32] with the
//     16-byte channel chunk XOR-swizzled by pixel (chunk ^ (pix >> 2) & 3) so the 16 lanes of a
//     fragment row read 16 different bank groups; conv2's k = tap*32 + ci;
//   * weights are split once on the host; each wave keeps its B fragments in registers for the
//     workgroup's lifetime (conv2: one 16-channel column block, 9 taps x 2 planes).
// Pooling is exact fp32 (max of the fp32 conv outputs after PReLU; bias and PReLU as the
// reference).  An operand that would leave the fp16 range (|pooled conv1| >= 2^14, or NaN) sets
// *ovf and the caller re-runs the candidates on the fp32 layer path.
#include <algorithm>
#include <cstdlib>

#include "common.hpp"
#include "mtcnn.hpp"
#include "mtcnn_dev.hpp"

namespace vtf {

namespace {

typedef __attribute__((ext_vector_type(8))) _Float16 h8;
typedef __attribute__((ext_vector_type(4))) _Float16 h4;
typedef __attribute__((ext_vector_type(4))) float f4;

constexpr int pool_side(int L) {
    // torch pooling_output_shape(L, 3, 0, 2, 1, ceil_mode=True)
    return ((L - 3 + 1) / 2 + 1 - 1) * 2 >= L ? (L - 3 + 1) / 2 : (L - 3 + 1) / 2 + 1;
}

template <int S, int C2, int PB1, int PB2, int MG>
struct Cfg {
    static constexpr int O1 = S - 2, P1 = pool_side(O1), O2 = P1 - 2, P2 = pool_side(O2);
    static constexpr int NF = C2 / 16, NW = NF * MG, NT = 64 * NW;
    static constexpr int CP = S + 2;  // crop plane side: conv1's padded taps (kx = 3, ky = 3) read zeros
    static constexpr int BR1 = 2 * PB1 + 1, BR2 = 2 * PB2 + 1;
    static constexpr int CROP = 2 * CP * CP * 4 * 2;   // [2][CP][CP][4] fp16
    static constexpr int RING1 = 32 * BR1 * O1 * 4;     // [32][BR1][O1] fp32
    static constexpr int POOL1 = 2 * P1 * P1 * 32 * 2;  // [2][P1*P1][32] fp16
    static constexpr int RING2 = BR2 * O2 * C2 * 4;     // [BR2][O2][C2] fp32
    static constexpr int STAGE = CROP + RING1 > RING2 ? CROP + RING1 : RING2;
    static constexpr int SMEM = POOL1 + STAGE;
};

__device__ inline h8 cat8(h4 lo, h4 hi) { return h8{lo[0], lo[1], lo[2], lo[3], hi[0], hi[1], hi[2], hi[3]}; }

__device__ inline void split_f16(float v, _Float16& x0, _Float16& x1) {
    x0 = (_Float16)v;
    x1 = (_Float16)((v - (float)x0) * 2048.f);
}

// pooled-conv1 element offset (halves) of pixel pix, channel c: 16-B chunk c>>3 swizzled by pixel
__device__ inline int p1_index(int pix, int c) { return pix * 32 + ((((c >> 3) ^ (pix >> 2)) & 3) << 3) + (c & 7); }

template <int S, int C2, int PB1, int PB2, int MG>
__global__ __launch_bounds__((Cfg<S, C2, PB1, PB2, MG>::NT)) void k_cand_fused(
    const void* __restrict__ sat, int pk, int H, int W, const float4* __restrict__ boxes, const int32_t* __restrict__ img,
    int64_t n, const _Float16* __restrict__ w1h, const float* __restrict__ b1, const float* __restrict__ a1,
    const _Float16* __restrict__ w2h, const float* __restrict__ b2, const float* __restrict__ a2,
    float* __restrict__ out, int32_t* __restrict__ err, int32_t* __restrict__ ovf, int dbg) {
    using C = Cfg<S, C2, PB1, PB2, MG>;
    constexpr int O1 = C::O1, P1 = C::P1, O2 = C::O2, P2 = C::P2, CP = C::CP, NT = C::NT, NW = C::NW;
    constexpr int BR1 = C::BR1, BR2 = C::BR2;
    constexpr int CPL = CP * CP * 4;      // crop plane (halves)
    constexpr int PPL = P1 * P1 * 32;     // pool1 plane (halves)
    __shared__ __attribute__((aligned(16))) char smem[C::SMEM];
    _Float16* pool1 = (_Float16*)smem;
    _Float16* crop = (_Float16*)(smem + C::POOL1);
    float* ring1 = (float*)(smem + C::POOL1 + C::CROP);
    float* ring2 = (float*)(smem + C::POOL1);  // aliases crop + ring1 (stage 2 only)

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6, lr = lane & 15, lg = lane >> 4;
    // conv2: this wave's 16-channel column block and M-fragment parity
    const int nf2 = wave % C::NF, mg = wave / C::NF;
    h8 b2f[9][2];
#pragma unroll
    for (int t = 0; t < 9; t++)
#pragma unroll
        for (int pl = 0; pl < 2; pl++)
            b2f[t][pl] = *(const h8*)(w2h + ((size_t)pl * C2 + nf2 * 16 + lr) * 288 + t * 32 + 8 * lg);
    const float cb2 = b2[nf2 * 16 + lr], ca2 = a2[nf2 * 16 + lr];
    int bad = 0;

    for (int64_t k = blockIdx.x; k < n; k += gridDim.x) {
        float* o = out + k * (P2 * P2 * C2);
        int y0, x0, hc, wc;
        if (!crop_rect(boxes[k], H, W, y0, x0, hc, wc)) {
            // the reference skips this box and then fails indexing (IndexError): flag it
            if (tid == 0) atomicAdd(err, 1);
            for (int i = tid; i < P2 * P2 * C2; i += NT) o[i] = 0.f;
            continue;  // uniform: every thread of the workgroup takes it
        }
        // ---- crop: S x S adaptive-pool bins from the SAT, split into the two planes
        const int64_t sk = (int64_t)img[k] * (H + 1) * (W + 1);
        for (int i = tid; i < CP * CP; i += NT) {
            const int r = i / CP, q = i - r * CP;
            h4 v0 = {0, 0, 0, 0}, v1 = {0, 0, 0, 0};
            if (r < S && q < S && !(dbg & 1)) {
                const int ys = (r * hc) / S, ye = ((r + 1) * hc + S - 1) / S;
                const int xs = (q * wc) / S, xe = ((q + 1) * wc + S - 1) / S;
                const int3 sm = sat_box_any(sat, pk, sk + x0, W + 1, y0 + ys, y0 + ye, xs, xe);
                const float c0 = bin_avg(sm.x, ye - ys, xe - xs);
                const float c1 = bin_avg(sm.y, ye - ys, xe - xs);
                const float c2 = bin_avg(sm.z, ye - ys, xe - xs);
                _Float16 h0, h1;
                split_f16(c0, h0, h1);
                v0[0] = h0;
                v1[0] = h1;
                split_f16(c1, h0, h1);
                v0[1] = h0;
                v1[1] = h1;
                split_f16(c2, h0, h1);
                v0[2] = h0;
                v1[2] = h1;
            }
            *(h4*)(crop + i * 4) = v0;
            *(h4*)(crop + CPL + i * 4) = v1;
        }
        __syncthreads();
        // ---- conv1 + PReLU in row bands into a ring of BR1 rows (a band's first row is the
        // previous band's last), then the ceil-mode 3x3/2 pool of the band into pool1 (split)
        for (int pr0 = 0; pr0 < P1; pr0 += PB1) {
            const int cr0 = 2 * pr0;
            const int r_lo = pr0 == 0 ? 0 : cr0 + 1;
            const int r_hi = min(cr0 + 2 * PB1, O1 - 1);
            const int npos = r_hi >= r_lo ? (r_hi - r_lo + 1) * O1 : 0;
            const int nfr = (npos + 15) / 16;
            for (int q = wave; q < ((dbg & 2) ? 0 : 2 * nfr); q += NW) {
                const int f = q >> 1, nf = q & 1;
                // conv1 B fragments of this 16-channel block (2 k-steps x 2 planes; L1-resident)
                h8 b1f[2][2];
#pragma unroll
                for (int s = 0; s < 2; s++)
#pragma unroll
                    for (int pl = 0; pl < 2; pl++)
                        b1f[s][pl] = *(const h8*)(w1h + (pl * 32 + nf * 16 + lr) * 64 + 32 * s + 8 * lg);
                const int p = min(f * 16 + lr, npos - 1);
                const int y = r_lo + p / O1, x = p % O1;
                f4 acc = {0.f, 0.f, 0.f, 0.f}, accx = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int s = 0; s < 2; s++) {
                    // k = 32 s + 8 lg + j: ky = 2 s + lg / 2, kx = 2 (lg & 1) + j / 4, c = j % 4
                    const int off = ((y + 2 * s + (lg >> 1)) * CP + x + 2 * (lg & 1)) * 4;
                    const h8 a0 = cat8(*(const h4*)(crop + off), *(const h4*)(crop + off + 4));
                    const h8 a1 = cat8(*(const h4*)(crop + CPL + off), *(const h4*)(crop + CPL + off + 4));
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b1f[s][0], acc, 0, 0, 0);
                    accx = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b1f[s][1], accx, 0, 0, 0);
                    accx = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b1f[s][0], accx, 0, 0, 0);
                }
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int qq = f * 16 + 4 * lg + i;
                    if (qq < npos) {
                        const int yq = r_lo + qq / O1, xq = qq % O1;
                        const float v = acc[i] + accx[i] * 0.00048828125f;
                        ring1[(nf * 16 + lr) * BR1 * O1 + (yq % BR1) * O1 + xq] = prelu(v + b1[nf * 16 + lr], a1[nf * 16 + lr]);
                    }
                }
            }
            __syncthreads();
            const int npr = (dbg & 4) ? 0 : min(PB1, P1 - pr0);
            for (int i = tid; i < npr * P1 * 32; i += NT) {
                const int c = i & 31, t = i >> 5;
                const int px = t % P1, py = pr0 + t / P1;
                float m = -3.402823466e38f;
                for (int dy = 0; dy < 3; dy++) {
                    const int yy = 2 * py + dy;
                    if (yy >= O1) break;
                    for (int dx = 0; dx < 3; dx++) {
                        const int xx = 2 * px + dx;
                        if (xx >= O1) break;
                        m = fmaxf(m, ring1[c * BR1 * O1 + (yy % BR1) * O1 + xx]);
                    }
                }
                bad |= !(fabsf(m) < 16384.f);
                _Float16 x0h, x1h;
                split_f16(m, x0h, x1h);
                const int e = p1_index(py * P1 + px, c);
                pool1[e] = x0h;
                pool1[PPL + e] = x1h;
            }
            __syncthreads();
        }
        // ---- conv2 + PReLU in row bands into ring2, then the 3x3/2 ceil pool straight to HBM
        for (int pr0 = 0; pr0 < P2; pr0 += PB2) {
            const int cr0 = 2 * pr0;
            const int r_lo = pr0 == 0 ? 0 : cr0 + 1;
            const int r_hi = min(cr0 + 2 * PB2, O2 - 1);
            const int npos = r_hi >= r_lo ? (r_hi - r_lo + 1) * O2 : 0;
            const int nfr = (npos + 15) / 16;
            for (int f = mg; f < ((dbg & 8) ? 0 : nfr); f += MG) {
                const int p = min(f * 16 + lr, npos - 1);
                const int y = r_lo + p / O2, x = p % O2;
                f4 acc = {0.f, 0.f, 0.f, 0.f}, accx = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
                for (int t = 0; t < 9; t++) {
                    const int pix = (y + t / 3) * P1 + x + t % 3;
                    const int e = pix * 32 + (((lg ^ (pix >> 2)) & 3) << 3);
                    const h8 a0 = *(const h8*)(pool1 + e);
                    const h8 a1 = *(const h8*)(pool1 + PPL + e);
                    acc = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b2f[t][0], acc, 0, 0, 0);
                    accx = __builtin_amdgcn_mfma_f32_16x16x32_f16(a0, b2f[t][1], accx, 0, 0, 0);
                    accx = __builtin_amdgcn_mfma_f32_16x16x32_f16(a1, b2f[t][0], accx, 0, 0, 0);
                }
#pragma unroll
                for (int i = 0; i < 4; i++) {
                    const int qq = f * 16 + 4 * lg + i;
                    if (qq < npos) {
                        const int yq = r_lo + qq / O2, xq = qq % O2;
                        const float v = acc[i] + accx[i] * 0.00048828125f;
                        ring2[((yq % BR2) * O2 + xq) * C2 + nf2 * 16 + lr] = prelu(v + cb2, ca2);
                    }
                }
            }
            __syncthreads();
            const int npr = (dbg & 16) ? 0 : min(PB2, P2 - pr0);
            for (int i = tid; i < npr * P2 * C2; i += NT) {
                const int c = i % C2, t = i / C2;
                const int px = t % P2, py = pr0 + t / P2;
                float m = -3.402823466e38f;
                for (int dy = 0; dy < 3; dy++) {
                    const int yy = 2 * py + dy;
                    if (yy >= O2) break;
                    for (int dx = 0; dx < 3; dx++) {
                        const int xx = 2 * px + dx;
                        if (xx >= O2) break;
                        m = fmaxf(m, ring2[((yy % BR2) * O2 + xx) * C2 + c]);
                    }
                }
                o[(py * P2 + px) * C2 + c] = m;
            }
            __syncthreads();
        }
    }
    if (__ballot(bad) && lane == 0) atomicOr(ovf, 1);
}

template <int S, int C2, int PB1, int PB2, int MG>
void launch_t(const void* sat, int pk, int H, int W, const float4* boxes, const int32_t* img, int64_t n,
              const CandFusedW& w, float* out, int32_t* err, int32_t* ovf, hipStream_t st) {
    using C = Cfg<S, C2, PB1, PB2, MG>;
    static_assert(C::SMEM <= 160 * 1024, "LDS budget");
    int dev = 0, cus = 256;
    VTF_HIP(hipGetDevice(&dev));
    VTF_HIP(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
    static int per_cu = 0;  // resident workgroups per CU (LDS and VGPR limits), once per instantiation
    if (!per_cu) {
        int b = 0;
        VTF_HIP(hipOccupancyMaxActiveBlocksPerMultiprocessor(&b, k_cand_fused<S, C2, PB1, PB2, MG>, C::NT, 0));
        per_cu = std::max(1, b);
    }
    const int64_t grid = std::min<int64_t>(n, (int64_t)cus * per_cu);
    static const int dbg = [] {  // phase-skip mask for profiling (VTF_CAND_DEBUG): 1 crop, 2 conv1,
        const char* e = std::getenv("VTF_CAND_DEBUG");  // 4 pool1, 8 conv2, 16 pool2
        return e ? std::atoi(e) : 0;
    }();
    k_cand_fused<S, C2, PB1, PB2, MG><<<(unsigned)grid, C::NT, 0, st>>>(sat, pk, H, W, boxes, img, n, w.w1h, w.b1, w.a1,
                                                                         w.w2h, w.b2, w.a2, out, err, ovf, dbg);
    VTF_HIP(hipGetLastError());
}

}  // namespace

int cand_fused_side(bool onet) { return onet ? Cfg<48, 64, 2, 2, 3>::P2 : Cfg<24, 48, 3, 4, 2>::P2; }

void launch_cand_fused(bool onet, const void* sat, int pk, int H, int W, const float4* boxes, const int32_t* img,
                       int64_t n, const CandFusedW& w, float* out, int32_t* err, int32_t* ovf, hipStream_t st) {
    if (n <= 0) return;
    if (onet)
        launch_t<48, 64, 2, 2, 3>(sat, pk, H, W, boxes, img, n, w, out, err, ovf, st);
    else
        launch_t<24, 48, 3, 4, 2>(sat, pk, H, W, boxes, img, n, w, out, err, ovf, st);
}

}  // namespace vtf

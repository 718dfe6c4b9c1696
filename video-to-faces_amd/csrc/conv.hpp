#pragma once
#include "common.hpp"

namespace vtf {

struct ConvParams {
    const void* in;      // NHWC [N,H,W,Cin], element type = precision
    const void* w;       // [Cout][KH*KW*Cin]
    void* out;           // NHWC, channel stride out_cstride, channel offset out_coff
    const float* bias;   // conv bias (or null)
    const float* alpha;  // BN scale (or null) -> v = v*alpha + beta
    const float* beta;
    const void* res;     // residual (NHWC, stride res_cstride) added after scale
    const float* prelu;  // per-channel PReLU slope (or null), applied last
    float scale;
    int relu;
    int gelu;            // exact erf GELU (ViT MLP, vit.py:37)
    int leaky;           // LeakyReLU(slope) (YOLO conv_unit 'lrelu_0.1', yolo.py:17-18)
    float slope;
    int res_post;        // residual added AFTER the activation (Darknet ResBlock y + x, yolo.py:28-31)
    int up2;             // write each output pixel to a 2x2 block of a (2*OH, 2*OW) tensor
                         // (F.interpolate(scale_factor=2) nearest, yolo.py:87,91)
    int res_up2;         // residual read at half resolution (nearest x2 upsample of a [N,OH/2,OW/2]
                         // map: the FPN top-down add, rcnn.py:26-27)
    int in_cstride;      // input channel stride (0 = Cin): read a channel slice of a concat buffer
    int out_f32;         // output is fp32 whatever the operand precision (detector heads)
    int f16x;            // fp32 operands on the fp16 matrix cores, split x = x0 + x1 * 2^-11 (fp32-grade
                         // products; the caller guarantees |operands| < 2^14, e.g. MTCNN's bounded nets)
    int* ovf;            // f16x mode: if set, an operand of magnitude >= 2^14 sets *ovf = 1 (the caller
                         // then re-runs in fp32: results are fp32-grade either way)
    int split_fp32;      // allow split-K in fp32 mode too (slice-order reduction: deterministic, but the
                         // summation order differs from the single pass; used where parity is a tolerance)
    int split;           // split-K factor (set by launch_conv; > 1: raw partial sums to ws)
    int group_m;         // XCD-aware tile order: M-tile group height (0 = plain blockIdx mapping; set by launch_conv)
    int xdbg;            // experiments only (built with -DVTF_CONV_XDBG=1, env VTF_CONV_XDBG, f16x mode):
                         // 1 = staging without the split arithmetic / range check, 2 = no operand loads
                         // (wrong results; timing only)
    float* ws;           // fp32 [split][M][Cout] partial sums (split-K only)
    int out_sp;          // output in the split-pair layout (gemm_x3.hpp; fp32 operand modes): the next
                         // layer's operand for conv_dma's split mode; a value beyond 2^14 sets *ovf
    int in_sp;           // input (and weights) in the split-pair layout: conv_dma split mode
    int s3;              // bf16x3 mode (conv_dma MODE 2): input, weights, residual and output (unless
                         // out_f32) in the split-triple layout (conv_dev.hpp)
    const void* zero;    // conv_dma: 16 zero bytes (the DMA source of padding / K-tail pieces; set by the launcher)
    int dp_tiles, tail_split, gx, gy;  // conv_dma work items (set by the launcher)
    int64_t M;           // N*OH*OW
    int N, H, W, Cin, OH, OW, Cout, KH, KW, sh, sw, ph, pw, K;
    int out_cstride, out_coff, res_cstride;
    // output channels >= n_split (n_split % 8 == 0; 0 = off) go to out2 [.., out2_cstride] at
    // channel out2_coff + (c - n_split): sibling 1x1 convs of one input run as one launch
    // (FaceNet branches) while each part lands in its own buffer
    int n_split;
    void* out2;
    int out2_cstride, out2_coff;
};

void launch_conv(const ConvParams& p, bool bf16, hipStream_t st);
// VTF_NO_SPLITK=1 (read per launch): no conv splits K into slices, so every output is one
// k-ordered MFMA chain (the fused FaceNet blocks' order: the bit-identity test's reference path)
bool splitk_disabled();
// LDS-DMA implicit-GEMM conv (conv_dma.hip): bf16 operands, or split-pair operands (in_sp, fp32-grade)
bool conv_dma_ok(const ConvParams& p);
// bf16 layer -> 0 k_conv, 1 conv_dma large tiles, 2 conv_dma 64 x 64 3-stage tiles (measured per shape)
int conv_dma_choice_bf16(const ConvParams& p);
void launch_conv_dma(const ConvParams& p, bool bf16, hipStream_t st);
// split-pair conv (bias + PReLU) fused with MaxPool2d(k, s, ceil_mode=True) writing the pooled map
// in split pairs (conv_dma.hip, k_conv_span_pool); returns false, launching nothing, when the
// shape does not fit the fused tiles (env VTF_CONV_SPAN_POOL=0: never)
bool launch_conv_span_pool(ConvParams p, int k, int s, void* pout, int& POH, int& POW, hipStream_t st);
void launch_maxpool(const void* in, int N, int H, int W, int C, void* out, int out_cstride, int out_coff, bool bf16,
                    hipStream_t st);
// torch MaxPool2d(k, s, ceil_mode) without padding, NHWC fp32; returns (OH, OW)
void launch_maxpool_ks(const float* in, int N, int H, int W, int C, int k, int s, bool ceil_mode, float* out,
                       int& OH, int& OW, hipStream_t st);
// the same pool with a split-pair output (gemm_x3.hpp; C % 8 == 0), range flag *ovf
void launch_maxpool_ks_sp(const float* in, int N, int H, int W, int C, int k, int s, bool ceil_mode, void* out, int& OH,
                          int& OW, int* ovf, hipStream_t st);
void launch_nchw_to_nhwc(const float* in, int N, int C, int H, int W, int Cp, void* out, bool bf16, hipStream_t st);
// scratch: N * (C + D) floats
void launch_facenet_head(const void* x, int N, int HW, int C, const float* w, const float* alpha, const float* beta,
                         int D, float* out, float* scratch, bool bf16, hipStream_t st);

}  // namespace vtf

/*
 * vtf.h — C ABI of libvtf_hip.so, the MI355X-native hot path of video-to-faces.
 *
 * The reference has no C ABI: its plugin surface is Python.  These entry
 * points are what that Python surface binds to (video-to-faces_amd/videotofaces/_native.py,
 * ctypes); each names the reference interface it replaces.  Conventions:
 *   - every call returns int status: 0 = ok, negative = error (message: vtf_last_error());
 *   - no exceptions cross the ABI; the caller owns every buffer it passes;
 *   - "d_" pointers are device (HBM) pointers, others are host pointers;
 *   - a handle is bound to one GPU and one HIP stream (vtf_*_set_stream) and is not
 *     thread-safe (the reference calls its models from one Python thread).
 */
#ifndef VTF_H
#define VTF_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define VTF_OK 0
#define VTF_E_ARG (-1)        /* bad argument (shape, null pointer, ...)           */
#define VTF_E_HIP (-2)        /* HIP runtime error                                 */
#define VTF_E_CAPACITY (-3)   /* output buffer too small; *out_total says how big  */
#define VTF_E_DEGENERATE (-4) /* reference crop loop would skip a box -> IndexError */
#define VTF_E_LIMIT (-5)      /* an internal size limit was exceeded               */

const char* vtf_last_error(void);
/* Free the library's per-stream scratch (box ops, dedupe, conv tail workspaces) of a HIP
 * stream the caller is about to destroy; waits for the stream.  Long-lived processes that
 * create streams per request call this so device memory stays bounded. */
int vtf_release_stream(void* hip_stream);
int vtf_version(void);

typedef struct vtf_mtcnn_s* vtf_mtcnn_t;
typedef struct vtf_facenet_s* vtf_facenet_t;
typedef struct vtf_vit_s* vtf_vit_t;
typedef struct vtf_yolo_s* vtf_yolo_t;
typedef struct vtf_group_s* vtf_group_t;
typedef struct vtf_rcnn_s* vtf_rcnn_t;

/* Box post-processing parameters (video_to_faces det_min_score, det_min_size, det_min_border,
 * det_scale, det_square; main.py:50-51), see vtf_boxes_to_crops. */
typedef struct vtf_box_params {
    float min_score;   /* compared in fp32 (numpy float32 vs Python float, NEP 50) */
    double min_size;   /* width or height below -> rejected */
    double min_border; /* 0 = no border check */
    double scale[4];   /* sx1, sx2, sy1, sy2 */
    int32_t square;
    int32_t adjust;    /* 1: adjust_boxes after filter_boxes (the pipeline); 0: filter_boxes only */
} vtf_box_params;

/* ---------------------------------------------------------------- MTCNN detector
 * Replaces RealMTCNN / MTCNN.forward (src/videotofaces/detectors/mtcnn.py:167-252,
 * 312-326), called by detection.py:131 `detout = model(frames)`.
 * params: fp32, the reference state_dict order minus num_batches_tracked
 *         (videotofaces/specs.py mtcnn_spec, 495,850 floats). */
int vtf_mtcnn_create(const float* params, int64_t n_params, int device, vtf_mtcnn_t* out);
int vtf_mtcnn_destroy(vtf_mtcnn_t h);
int vtf_mtcnn_set_stream(vtf_mtcnn_t h, void* hip_stream);

/* frames: uint8 BGR, frame b pixel (y,x) channel c at frames[b*frame_stride + y*row_stride
 * + x*3 + c] (a borrowed, possibly non-contiguous view, detection.py:114-116).
 * frames_on_device: 1 if `frames` is a device pointer.
 * Output (host): boxes [total,5] (x1,y1,x2,y2,score), landmarks [total,5,2] ((x,y) per point, as
 * mtcnn.py:239 stacks them; may be NULL), counts[B]; per image in reference order.  If total > cap nothing is
 * written, *out_total is set and VTF_E_CAPACITY returned. */
int vtf_mtcnn_detect(vtf_mtcnn_t h, const uint8_t* frames, int frames_on_device, int B, int H, int W,
                     int64_t frame_stride, int64_t row_stride, double min_face_size,
                     float* out_boxes, float* out_landmarks, int32_t* out_counts, int64_t cap,
                     int64_t* out_total);

/* detect + box post-processing with nothing on the host but the counts: the detector's rows
 * stay in HBM and go through vtf_boxes_to_crops (detection.py:131-145).  frames as above;
 * d_crops / out_frame_counts / cap / out_n as in vtf_boxes_to_crops. */
int vtf_mtcnn_detect_crops(vtf_mtcnn_t h, const uint8_t* frames, int frames_on_device, int B, int H, int W,
                           int64_t frame_stride, int64_t row_stride, double min_face_size,
                           const vtf_box_params* params, int32_t frame_offset, int32_t* d_crops,
                           int32_t* out_frame_counts, int64_t cap, int64_t* out_n);

/* Per-stage counters of the last detect call: [0] levels, [1] stage-1 candidates (all
 * levels), [2] after per-level NMS, [3] after cross-level NMS (= stage-2 proposals),
 * [4] stage-2 passing, [5] after stage-2 NMS (= stage-3 refinements), [6] stage-3 passing,
 * [7] final faces. */
int vtf_mtcnn_stats(vtf_mtcnn_t h, int64_t* out8);

/* Parity introspection (tests): enable = 1 / 0 turns recording of the stage-1 candidate set on /
 * off for later detect calls (-1 leaves it), then the last call's stage-1 keys -- (level << 32 |
 * (b * ph + y) * pw + x) of every cell with p >= 0.6, ascending = the reference's per-level
 * nonzero() order (mtcnn.py:183-186) -- are copied to out (up to cap) and their count to *out_n. */
int vtf_mtcnn_stage1_keys(vtf_mtcnn_t h, int enable, uint64_t* out, int64_t cap, int64_t* out_n);

/* Kernel timing of the dominant kernel (fused pyramid+PNet) with HIP events recorded on the
 * handle's stream around each launch.  enable=1 resets and starts accumulating; the call
 * returns the totals so far: elapsed ms, launches, algorithmic FLOPs (2*MAC of conv1-3 and
 * the heads over every pyramid level) and frames. */
int vtf_mtcnn_profile(vtf_mtcnn_t h, int enable, double* out_ms, int64_t* out_launches, double* out_flops,
                      int64_t* out_frames);

/* Parity entry points (device pointers, handle stream).
 * Fused MTCNN._resample + PNet for one pyramid level (mtcnn.py:150-151, 27-38):
 * d_prob [B,ph,pw], d_reg [B,4,ph,pw] with ph = ceil((lh-2)/2)-4. */
int vtf_mtcnn_pnet_level(vtf_mtcnn_t h, const uint8_t* d_frames, int B, int H, int W, int64_t frame_stride,
                         int64_t row_stride, int lh, int lw, float* d_prob, float* d_reg);
/* MTCNN._resample of the preprocessed frames (mtcnn.py:133-139,150-151): d_out [B,3,lh,lw]. */
int vtf_mtcnn_resample(vtf_mtcnn_t h, const uint8_t* d_frames, int B, int H, int W, int64_t frame_stride,
                       int64_t row_stride, int lh, int lw, float* d_out);
/* RNet / ONet on given fp32 NCHW inputs (mtcnn.py:58-76, 101-121). */
int vtf_mtcnn_rnet(vtf_mtcnn_t h, const float* d_in, int64_t n, float* d_reg, float* d_prob);
int vtf_mtcnn_onet(vtf_mtcnn_t h, const float* d_in, int64_t n, float* d_reg, float* d_lm, float* d_prob);

/* ---------------------------------------------------------------- box post-processing
 * process_frames_batch steps 2-5 (src/videotofaces/detection.py:133-145) on device:
 * filter_boxes (detection.py:174-217, with check_box 165-171), adjust_boxes (220-262) and the
 * (frame, face) flatten of get_crops (161-162).  Parameters as video_to_faces passes them
 * (main.py:50-51): det_min_score, det_min_size, det_min_border, det_scale (sx1, sx2, sy1, sy2),
 * det_square. */

/* d_rows: device fp32 [n,5] (x1,y1,x2,y2,score) grouped by frame, counts: host int32 [B] rows per
 * frame (negative = frame absent from the detector output: no crops).  Writes device int32
 * d_crops [m,5] (frame_offset + frame, x1, y1, x2, y2) in row order, d_src [m] (source row, may be
 * NULL), host out_frame_counts [B] (may be NULL) and *out_n = m.  VTF_E_CAPACITY when the rows
 * exceed cap (then *out_n = rows, nothing written). */
int vtf_boxes_to_crops(const float* d_rows, const int32_t* counts, int B, int H, int W, const vtf_box_params* params,
                       int32_t frame_offset, int32_t* d_crops, int32_t* d_src, int32_t* out_frame_counts,
                       int64_t cap, int64_t* out_n, void* hip_stream);

/* ---------------------------------------------------------------- box ops
 * torchvision.ops.batched_nms as called at mtcnn.py:196,205,219 and
 * detectors/operations/post.py:8: d_boxes [n,4] fp32, d_scores [n], d_idxs [n] int64.
 * Writes keep indices (int64, score-descending) to d_keep and their count to *out_nkeep. */
int vtf_batched_nms(const float* d_boxes, const float* d_scores, const int64_t* d_idxs, int64_t n,
                    double iou_threshold, int64_t* d_keep, int64_t* out_nkeep, void* hip_stream);

/* MTCNN._nms_vectorized(boxes, scores, classes, thr, 'Min') with chain suppression
 * (mtcnn.py:273-309, called at 242): rows sorted by descending score (ties in index order:
 * the reference's argsort is unstable there), a row is dropped when ANY earlier row of the same
 * class overlaps it with intersection-over-minimum (+1 pixel widths) > thr (fp32).
 * d_boxes [n,4] fp32, d_scores [n], d_classes [n] int32 -> d_keep int64 (kept rows in that
 * order), *out_nkeep. */
int vtf_iom_nms(const float* d_boxes, const float* d_scores, const int32_t* d_classes, int64_t n, float thr,
                int64_t* d_keep, int64_t* out_nkeep, void* hip_stream);

/* ---------------------------------------------------------------- FaceNet encoder
 * Replaces FaceNet / InceptionResnetV1 (src/videotofaces/encoders/facenet.py:123-183),
 * called by grouping.py:37 `xk = model(images)`.
 * precision: 0 = fp32 (parity mode), 1 = bf16 activations/weights with fp32 accumulation. */
int vtf_facenet_create(const float* params, int64_t n_params, int device, int precision, vtf_facenet_t* out);
int vtf_facenet_destroy(vtf_facenet_t h);
int vtf_facenet_set_stream(vtf_facenet_t h, void* hip_stream);
/* Encoder on blob input: d_x [N,3,160,160] fp32 NCHW RGB (cv2.dnn.blobFromImages output,
 * facenet.py:179) -> d_emb [N,512] fp32, L2-normalised. */
int vtf_facenet_forward(vtf_facenet_t h, const float* d_x, int64_t N, float* d_emb);
/* Crop + resize + normalise faces straight from device frames (blobFromImages(1/128,
 * 160x160, 127.5, swapRB) on each crop, INTER_LINEAR uint8), then encode.
 * d_frames: F device frames as in vtf_mtcnn_detect; crops int32 [N,5] (frame index, x1, y1,
 * x2, y2) in frame pixels (detection.py:161-162 get_crops slices), a host array (validated:
 * 0 <= frame < F, non-empty slice inside the frame, else VTF_E_ARG) or, with crops_on_device,
 * a device array such as vtf_*_detect_crops writes (read by the kernel; an invalid rectangle
 * encodes a zero image instead of reading outside the frames). */
int vtf_facenet_encode_crops(vtf_facenet_t h, const uint8_t* d_frames, int F, int H, int W, int64_t frame_stride,
                             int64_t row_stride, const int32_t* crops, int crops_on_device, int64_t N,
                             float* d_emb);
/* Blob of uint8 BGR crops (cv2.dnn.blobFromImages, INTER_LINEAR, swapRB): d_out [N,3,S,S].
 * out = (resized_u8 - mean) * scale.  d_crops: device int32 [N,5] into F frames. */
int vtf_blob_from_crops(const uint8_t* d_frames, int F, int H, int W, int64_t frame_stride, int64_t row_stride,
                        const int32_t* d_crops, int64_t N, int S, float mean, float scale, float* d_out,
                        void* hip_stream);

/* ---------------------------------------------------------------- ViT encoder
 * Replaces ViT / AnimeVIT (src/videotofaces/encoders/vit.py:80-146), called by grouping.py:37.
 * dim 768 / depth 12 (B16) or 1024 / 24 (L16); params in the reference state_dict order
 * (specs.py vit_spec).  fp32 or guarded split-fp16 (vtf_vit_set_precision). */
int vtf_vit_create(const float* params, int64_t n_params, int dim, int depth, int device, vtf_vit_t* out);
int vtf_vit_destroy(vtf_vit_t h);
int vtf_vit_set_stream(vtf_vit_t h, void* hip_stream);
/* GEMM operand mode: 0 = fp32 MFMA (default); 2 = fp32 operands split into two fp16 parts on the
 * fp16 matrix cores (fp32-grade products), guarded: an operand >= 2^14 re-runs the forward in fp32. */
int vtf_vit_set_precision(vtf_vit_t h, int mode);
/* d_x [N,3,128,128] fp32 blob (blobFromImages(1/127.5, 128x128, 127.5, swapRB)) -> d_emb [N,dim]
 * (LayerNorm of the CLS token, not L2-normalised). */
int vtf_vit_forward(vtf_vit_t h, const float* d_x, int64_t N, float* d_emb);
/* crops as in vtf_facenet_encode_crops, resized to 128x128 (vit.py:141). */
int vtf_vit_encode_crops(vtf_vit_t h, const uint8_t* d_frames, int F, int H, int W, int64_t frame_stride,
                         int64_t row_stride, const int32_t* crops, int crops_on_device, int64_t N, float* d_emb);

/* fp32-grade GEMM on the fp16 matrix cores (the split-fp16 ViT Linear layers, vit.py:29-37):
 * out[M,N] = a[M,K] b[N,K]^T (+ bias[N]); device fp32 row-major operands, split on device into
 * x0 + x1 * 2^-11 fp16 pairs (|x| < 2^14 required: VTF_E_ARG otherwise).  K % 32 == 0, N % 8 == 0.
 * Stream-ordered; returns after the stream is synchronised. */
int vtf_gemm_split(const float* d_a, const float* d_b, int64_t M, int N, int K, const float* d_bias, float* d_out,
                   void* hip_stream);

/* ---------------------------------------------------------------- grouping
 * remove_dupes_overall 'enc' branch (dupes.py:51-68 with sklearn cosine_distances):
 * for each row i, min and argmin over j < i of clip(1 - cos(X_i, X_j), 0, 2); row 0 gets
 * 10000 / 0 (the reference's masked diagonal).  d_X [N,D] fp32 -> d_min [N], d_arg [N]. */
int vtf_cosine_dedupe(const float* d_X, int64_t N, int64_t D, float* d_min, int64_t* d_arg, void* hip_stream);
/* The same for rows [row_begin, row_end) only (a rank's shard of the lower triangle, SURVEY.md
 * §8e): row_begin a multiple of 128, row_end a multiple of 128 or N; d_min / d_arg hold
 * row_end - row_begin entries.  Rows at or after row_end are not read. */
int vtf_cosine_dedupe_rows(const float* d_X, int64_t N, int64_t D, int64_t row_begin, int64_t row_end, float* d_min,
                           int64_t* d_arg, void* hip_stream);
/* classify (grouping.py:50-55): min / first argmin over c of sklearn cosine_distances(X, R)[i, c]
 * in sklearn's own bits (normalize; X_n @ R_n.T as numpy's OpenBLAS sgemm / sgemv / sdot orders;
 * clip(1 - G, 0, 2)).  d_X [N,D], d_R [C,D] fp32 -> d_min [N] fp32, d_arg [N] int64. */
int vtf_cosine_classify(const float* d_X, int64_t N, const float* d_R, int64_t C, int64_t D, float* d_min,
                        int64_t* d_arg, void* hip_stream);
/* the full matrix dist = cosine_distances(X, R) of classify (grouping.py:51) in the same bits:
 * d_dist [N,C] fp32 (the per-class distances of log_classification.csv, grouping.py:58-64). */
int vtf_cosine_distances_xr(const float* d_X, int64_t N, const float* d_R, int64_t C, int64_t D, float* d_dist,
                            void* hip_stream);

/* ---------------------------------------------------------------- hash dedupe
 * dupes.ahash (dupes.py:11-15) of N face crops of device frames (frames as in
 * vtf_mtcnn_detect (F frames), crops host int32 [N,5] = frame, x1, y1, x2, y2 as get_crops slices them
 * (validated as in vtf_facenet_encode_crops),
 * detection.py:161-162): out_hashes host uint64 [N], bit k = 8x8 thumbnail pixel k (row-major)
 * > mean.  cvtColor(BGR2GRAY) + resize INTER_LINEAR restated from OpenCV's fixed point. */
int vtf_ahash_crops(const uint8_t* d_frames, int F, int H, int W, int64_t frame_stride, int64_t row_stride,
                    const int32_t* crops, int64_t N, uint64_t* out_hashes, void* hip_stream);
/* remove_dupes_overall('hash') distances (dupes.py:55-64): for row i, min and first argmin over
 * j < i of popcount(h_i ^ h_j); row 0 -> 10000, 0.  d_hashes uint64 [N] -> d_min int32 [N],
 * d_arg int64 [N]. */
int vtf_hamming_dedupe(const uint64_t* d_hashes, int64_t N, int32_t* d_min, int64_t* d_arg, void* hip_stream);

/* ---------------------------------------------------------------- video frames
 * The decode side of process_video (src/videotofaces/detection.py:68-111, which hands the
 * detector cv2.VideoCapture / decord BGR frames [B,H,W,3]): planar YUV frames in HBM (as a
 * YUV4MPEG2 stream stores them: Y [H][W], then U and V planes of the chroma size) -> uint8 BGR.
 * d_yuv: n frames at in_frame_stride bytes; chroma 420 / 422 / 444 / 400 (mono, U = V = 128);
 * full_range 0 = BT.601 limited range (OpenCV's COLOR_YUV2BGR_I420 integer transform), 1 = full
 * range; chroma sampled nearest.  d_bgr: [n][H][W][3] at the given frame / row strides (bytes).
 * Asynchronous on hip_stream. */
int vtf_yuv_to_bgr(const uint8_t* d_yuv, int64_t n, int H, int W, int chroma, int full_range, int64_t in_frame_stride,
                   uint8_t* d_bgr, int64_t out_frame_stride, int64_t out_row_stride, void* hip_stream);

/* ---------------------------------------------------------------- YOLOv3 detector
 * Replaces RealYOLO / YOLOv3.forward (src/videotofaces/detectors/yolo.py:131-191), called by
 * detection.py:131 `detout = model(frames)`.
 * params: fp32, reference state_dict order minus num_batches_tracked (specs.py yolo_spec,
 *         61,576,342 floats).  precision 0 = fp32 (parity), 1 = bf16 operands/activations. */
int vtf_yolo_create(const float* params, int64_t n_params, int device, int precision, vtf_yolo_t* out);
int vtf_yolo_destroy(vtf_yolo_t h);
int vtf_yolo_set_stream(vtf_yolo_t h, void* hip_stream);
/* frames as in vtf_mtcnn_detect.  Output (host): boxes [total,4] (x1,y1,x2,y2 in frame
 * pixels, unclamped), scores [total], counts[B] (<= 100 each); per image in the reference's
 * order (score desc).  Classes are all 0 (num_classes=1).  VTF_E_CAPACITY as in mtcnn. */
int vtf_yolo_detect(vtf_yolo_t h, const uint8_t* frames, int frames_on_device, int B, int H, int W,
                    int64_t frame_stride, int64_t row_stride, float* out_boxes, float* out_scores,
                    int32_t* out_counts, int64_t cap, int64_t* out_total);
/* detect + box post-processing on device, as vtf_mtcnn_detect_crops. */
int vtf_yolo_detect_crops(vtf_yolo_t h, const uint8_t* frames, int frames_on_device, int B, int H, int W,
                          int64_t frame_stride, int64_t row_stride, const vtf_box_params* params,
                          int32_t frame_offset, int32_t* d_crops, int32_t* out_frame_counts, int64_t cap,
                          int64_t* out_n);
/* resize_cv2 keep-ratio size (prep.py:71-73) and the x32 padded net input: {h, w, Hp, Wp}. */
int vtf_yolo_input_size(int H, int W, int* out4);
/* Parity entries.  letterbox: preprocess (prep.py:12-92) -> d_out NHWC fp32 [B,Hp,Wp,8]
 * (channels 3..7 zero).  net: d_x NCHW fp32 [B,3,Hp,Wp] -> pred maps NHWC fp32
 * [B,Hp/32,Wp/32,18], [B,Hp/16,Wp/16,18], [B,Hp/8,Wp/8,18] (yolo.py:143-145).
 * postprocess: the maps of frames of size HxW -> detect's outputs (yolo.py:146-147). */
int vtf_yolo_letterbox(vtf_yolo_t h, const uint8_t* d_frames, int B, int H, int W, int64_t frame_stride,
                       int64_t row_stride, float* d_out);
int vtf_yolo_net(vtf_yolo_t h, const float* d_x, int B, int Hp, int Wp, float* d_map0, float* d_map1,
                 float* d_map2);
int vtf_yolo_postprocess(vtf_yolo_t h, const float* d_map0, const float* d_map1, const float* d_map2, int B,
                         int H, int W, float* out_boxes, float* out_scores, int32_t* out_counts, int64_t cap,
                         int64_t* out_total);
/* Conv-stack timing (HIP events around the 75 conv launches of each detect/net call):
 * accumulated ms, launches, algorithmic FLOPs and frames since the last call; enable != 0
 * turns timing on for the following calls. */
int vtf_yolo_profile(vtf_yolo_t h, int enable, double* out_ms, int64_t* out_launches, double* out_flops,
                     int64_t* out_frames);

/* ---------------------------------------------------------------- Faster R-CNN detector
 * Replaces AnimeFRCNN / FasterRCNN.forward (src/videotofaces/detectors/rcnn.py:127-177),
 * called by detection.py:131 `detout = model(frames)` for style='anime'.
 * params: fp32, reference state_dict order minus num_batches_tracked (specs.py rcnn_spec,
 *         41,401,301 floats).  precision 0 = fp32 (parity), 1 = bf16 operands/activations. */
int vtf_rcnn_create(const float* params, int64_t n_params, int device, int precision, vtf_rcnn_t* out);
int vtf_rcnn_destroy(vtf_rcnn_t h);
int vtf_rcnn_set_stream(vtf_rcnn_t h, void* hip_stream);
/* frames as in vtf_mtcnn_detect.  Output (host): boxes [total,4] (x1,y1,x2,y2 in frame pixels),
 * scores [total], counts[B] (<= 100 each), per image in the reference's order (score desc).
 * counts[b] = -1 for images after the last one holding an RPN proposal: the reference returns
 * only max(imidx)+1 lists (rcnn.py:111).  Classes are all 0.  VTF_E_CAPACITY as in mtcnn. */
int vtf_rcnn_detect(vtf_rcnn_t h, const uint8_t* frames, int frames_on_device, int B, int H, int W,
                    int64_t frame_stride, int64_t row_stride, float* out_boxes, float* out_scores,
                    int32_t* out_counts, int64_t cap, int64_t* out_total);
/* detect + box post-processing on device, as vtf_mtcnn_detect_crops (frames past the last
 * proposal image produce no crops, as the reference's shorter detout list does). */
int vtf_rcnn_detect_crops(vtf_rcnn_t h, const uint8_t* frames, int frames_on_device, int B, int H, int W,
                          int64_t frame_stride, int64_t row_stride, const vtf_box_params* params,
                          int32_t frame_offset, int32_t* d_crops, int32_t* out_frame_counts, int64_t cap,
                          int64_t* out_n);
/* resize_cv2 keep-ratio size for resize=(800, 1333) (prep.py:71-74) and the x32 padded net
 * input: {h, w, Hp, Wp}. */
int vtf_rcnn_input_size(int H, int W, int* out4);
/* Parity entries.  preprocess (prep.py:12-92, imagenet mean/std) -> d_out NHWC fp32
 * [B,Hp,Wp,8] (channels 3..7 zero).  rpn_heads: body + FPN + RPN head on d_x NCHW fp32
 * [B,3,Hp,Wp] -> per level l (strides 4..64) NHWC fp32 [B,h_l,w_l,15]: 3 logits
 * (RegionProposalNetwork.log) then 3 x 4 deltas (.reg), rcnn.py:42-47. */
int vtf_rcnn_preprocess(vtf_rcnn_t h, const uint8_t* d_frames, int B, int H, int W, int64_t frame_stride,
                        int64_t row_stride, float* d_out);
int vtf_rcnn_rpn_heads(vtf_rcnn_t h, const float* d_x, int B, int Hp, int Wp, float* d_head0, float* d_head1,
                       float* d_head2, float* d_head3, float* d_head4);
/* RPN proposals of the last detect call (rcnn.py:82): host [n,5] (image, x1, y1, x2, y2). */
int vtf_rcnn_proposals(vtf_rcnn_t h, float* out, int64_t cap, int64_t* out_n);
/* RegionProposalNetwork.forward after the heads (rcnn.py:49-82: per-level top-1000, decode,
 * clamp, remove_small, batched_nms(0.7) by (image, level), top-1000 per image) on given head maps
 * (NHWC fp32 as vtf_rcnn_rpn_heads writes them) of a B x Hp x Wp input whose images are
 * h_used x w_used: host out [n,5] (image, x1, y1, x2, y2).  The integer path (top-k, NMS keep
 * sets) can so be checked on identical inputs. */
int vtf_rcnn_rpn_proposals(vtf_rcnn_t h, const float* d_head0, const float* d_head1, const float* d_head2,
                           const float* d_head3, const float* d_head4, int B, int Hp, int Wp, int h_used, int w_used,
                           float* out, int64_t cap, int64_t* out_n);
/* torchvision.ops.roi_align(fmap, rois, (7,7), spatial_scale, sampling_ratio=0, aligned=True)
 * as roi.py:31 calls it: d_fmap NHWC fp32 [N,H,W,C], d_rois fp32 [R,5] (image, x1, y1, x2, y2)
 * -> d_out NHWC fp32 [R,7,7,C]. */
int vtf_roi_align(const float* d_fmap, int N, int H, int W, int C, const float* d_rois, int64_t R,
                  float spatial_scale, float* d_out, void* hip_stream);
/* Timing of the body + FPN + RPN-head conv stack, as vtf_yolo_profile. */
int vtf_rcnn_profile(vtf_rcnn_t h, int enable, double* out_ms, int64_t* out_launches, double* out_flops,
                     int64_t* out_frames);

/* ---------------------------------------------------------------- grouping: K-means, scores
 * Replace the sklearn calls of cluster_faces (src/videotofaces/grouping.py:92-120):
 * KMeans(n_clusters=k, random_state, n_init='auto').fit(X), silhouette_score,
 * calinski_harabasz_score, davies_bouldin_score.  The host mirror (videotofaces/kmeans.py)
 * keeps sklearn's scalar control flow; these are its device passes.  All device arrays are
 * row-major, X float32 [N,D]. */
int vtf_group_create(int device, vtf_group_t* out);
int vtf_group_destroy(vtf_group_t h);
int vtf_group_set_stream(vtf_group_t h, void* hip_stream);
/* X.mean(axis=0), np.var(X, axis=0) (numpy's sequential fp32 axis-0 sums) and, if d_Xc is
 * not NULL, the centred copy X - mean (KMeans.fit, sklearn/cluster/_kmeans.py:1479-1481). */
int vtf_colstats(vtf_group_t h, const float* d_X, int64_t N, int64_t D, float* d_Xc, float* d_mean, float* d_var);
/* k-means++ distances (_kmeans.py:_kmeans_plusplus): d_out [T,N] = squared euclidean
 * distances of rows[0..T) (host int64 indices) to every row, sklearn's float64-upcast
 * formula rounded to fp32 and clipped at 0.  T <= 16. */
int vtf_sqdist_rows(vtf_group_t h, const float* d_X, int64_t N, int64_t D, const int64_t* rows, int T, float* d_out);
/* One Lloyd iteration (_k_means_lloyd.pyx lloyd_iter_chunked_dense): labels (in/out, int32)
 * from centers [k,D]; if d_sums: per-cluster sums [k,D] in sklearn's one-thread order
 * (sequential fp32 over the cluster's rows in row order, _update_chunk_dense) and weights
 * [k] (counts).  *out_changed = number of labels that changed.  k <= 64, N < 2^24. */
int vtf_kmeans_step(vtf_group_t h, const float* d_X, int64_t N, int64_t D, const float* d_centers, int k,
                    int32_t* d_labels, float* d_sums, float* d_weights, int64_t* out_changed);
/* _average_centers + _center_shift: sums -> centers in place, shift[k] = |new - old|. */
int vtf_kmeans_average(vtf_group_t h, float* d_sums, const float* d_weights, const float* d_centers_old, int k,
                       int64_t D, float* d_shift);
/* ((X - centers[labels])**2).sum(1) (empty-cluster relocation, _k_means_common.pyx). */
int vtf_center_dist(vtf_group_t h, const float* d_X, int64_t N, int64_t D, const float* d_centers,
                    const int32_t* d_labels, float* d_out);
/* pairwise_distances(X) euclidean [N,N] fp32 (float64-upcast, sqrt, zero diagonal). */
int vtf_pairwise_euclidean(vtf_group_t h, const float* d_X, int64_t N, int64_t D, float* d_out);
/* silhouette_samples from the distance matrix; labels encoded 0..k-1, freq int64 [k]. */
int vtf_silhouette_samples(vtf_group_t h, const float* d_D, int64_t N, const int32_t* d_labels, int k,
                           const int64_t* d_freq, float* d_sil);
/* silhouette_samples (sklearn/metrics/cluster/_unsupervised.py:203-315, called by
 * silhouette_score at grouping.py:105) of M label sets at once, for rows [row_begin, row_end)
 * only -- a rank's shard -- and without the N x N matrix (O(N*D) memory): d_labels uint8
 * [M][N] encoded 0..k_m-1, ks host int32 [M] (2 <= k_m, sum k_m <= 160 per call), freq host
 * int64 [sum k_m] (cluster sizes, set after set), d_sil float32 [M][row_end - row_begin].
 * Replaces vtf_pairwise_euclidean + vtf_silhouette_samples for the sweep. */
int vtf_silhouette_sweep(vtf_group_t h, const float* d_X, int64_t N, int64_t D, int64_t row_begin, int64_t row_end,
                         const uint8_t* d_labels, int M, const int32_t* ks, const int64_t* freq, float* d_sil);
/* Per-cluster float64 sums [k,D], sum of |x|^2 [k] and counts [k] (calinski_harabasz). */
int vtf_cluster_sums(vtf_group_t h, const float* d_X, int64_t N, int64_t D, const int32_t* d_labels, int k,
                     double* d_sums, double* d_sqnorm, int64_t* d_counts);
/* dsum[c] = sum over members of |x - centroid_c| in float64 (davies_bouldin intra_dists). */
int vtf_cluster_dist(vtf_group_t h, const float* d_X, int64_t N, int64_t D, const int32_t* d_labels, int k,
                     const double* d_centroids, double* d_dsum);

#ifdef __cplusplus
}
#endif
#endif /* VTF_H */

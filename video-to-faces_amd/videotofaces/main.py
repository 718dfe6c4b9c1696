"""The public API: video_to_faces() (drop-in for src/videotofaces/main.py:13-82).

Same keyword arguments, defaults, validation messages and stage order as the reference:
detection (frames -> detector -> box filter/adjust -> hash dedupe -> face JPEGs) then grouping
(JPEGs -> encoder -> embedding dedupe -> K-means clustering or classification).  Every model
and every all-pairs / K-means pass runs in libvtf_hip.so.  Additions, all opt-in:
  * input_path may be a .npy file or a uint8 array [F,H,W,3] of frames (fps 1) -- video
    decode needs OpenCV, which this image lacks (decode is a later row);
  * decoupled=True lifts the style <-> model coupling (prep.py:39-44), e.g. det_model='yolo'
    with enc_model='vit_l' (BASELINE config 5);
  * det_precision / enc_precision select the operand mode of YOLO / R-CNN and FaceNet / ViT:
    'fp32' (default, fp32 MFMA: the parity mode), 'bf16' (bf16 operands; FaceNet, YOLO, R-CNN)
    or 'f16x' (fp32 operands split into two fp16 parts, fp32-grade products; ViT).  The
    reference-default paths (det_model / enc_model 'default') keep the reference classes'
    defaults.
"""
import os.path as osp

import torch

from . import prep


def get_detector(style, det_model, device, precision='fp32'):
    from .detection import get_detector_model
    if det_model in ('default', None):
        return get_detector_model(style, det_model, device)
    if det_model == 'mtcnn':
        from .detectors.mtcnn import RealMTCNN
        return RealMTCNN(device)
    if det_model == 'yolo':
        from .detectors.yolo import RealYOLO
        return RealYOLO(device, precision=precision)
    from .detectors.rcnn import AnimeFRCNN
    return AnimeFRCNN(device, precision=precision)


def get_encoder(style, enc_model, device, precision='fp32'):
    from .grouping import get_encoder_model
    if enc_model in ('default', None):
        return get_encoder_model(style, enc_model, device)
    if enc_model.startswith('vit'):
        from .encoders.vit import AnimeVIT
        return AnimeVIT(device, enc_model[-1] == 'l', precision=precision)
    from .encoders.facenet import FaceNet
    return FaceNet(device, enc_model.split('_')[1] == 'casia', precision=precision)


def video_to_faces(input_path=None, input_ext=None,
                   mode='full', style='anime', device=None,
                   out_dir=None, out_prefix='', resize_to=None,
                   save_frames=False, save_rejects=False, save_dupes=False,
                   video_step=1, video_fragment=None, video_area=None, video_reader='opencv',
                   det_model='default', det_batch_size=4, det_min_score=0.4, det_min_size=50,
                   det_min_border=5, det_scale=(1.5, 1.5, 2.2, 1.2), det_square=True,
                   hash_thr=8,
                   enc_model='default', enc_batch_size=16, enc_area=None,
                   group_mode='clustering', clusters=None, clusters_save_all=False,
                   ref_dir=None, random_state=0, group_log=True,
                   enc_dup_thr=0.25, enc_oth_thr=0.9,
                   _test_enc=False, _test_exclude_other=False,
                   decoupled=False, det_precision='fp32', enc_precision='fp32'):
    from .detection import detect_faces
    from .dupes import remove_dupes_overall
    from .grouping import encode_faces, cluster_faces, classify_faces
    if not prep.validate_args(mode, input_path, out_dir, style, group_mode, video_reader, det_model, enc_model,
                              decoupled):
        return
    if _test_enc:
        raise NotImplementedError('_test_enc needs a labels.txt ground truth (grouping.py:140-155)')
    in_memory = input_path is not None and not isinstance(input_path, str)
    if det_model == 'default':
        det_model = 'rcnn' if style == 'anime' else 'yolo'
    if enc_model == 'default':
        enc_model = 'vit_b' if style == 'anime' else 'facenet_vgg'
    if not out_dir:
        if in_memory:
            print('ERROR: out_dir is required with in-memory frames')
            return
        out_dir = input_path if osp.isdir(input_path) else osp.dirname(osp.abspath(input_path))
    if not device:
        device = torch.device('cuda:0')
    if mode != 'detection' and group_mode == 'clustering':
        clusters = prep.get_clusters(clusters)
        if not clusters:
            return
    if mode != 'detection' and group_mode == 'classification':
        refs = prep.get_class_ref(ref_dir, out_dir)
        if not refs:
            return
    imgpaths = None
    if mode == 'grouping':
        imgpaths = prep.get_paths_for_grouping(out_dir)
        if not imgpaths:
            return
    if mode in ('full', 'detection'):
        files = [input_path] if in_memory else prep.get_video_list(input_path, input_ext)
        if not len(files):
            return
        vid_params = (video_step, video_fragment, video_area, video_reader)
        det_params = (det_batch_size, det_min_score, det_min_size, det_min_border, det_scale, det_square)
        save_params = (out_dir, out_prefix, resize_to, save_frames, save_rejects, save_dupes)
        detector = get_detector(style, det_model, device, det_precision)
        imgpaths = detect_faces(files, detector, vid_params, det_params, save_params, hash_thr)
    if mode in ('full', 'grouping') and imgpaths:
        encoder = get_encoder(style, enc_model, device, enc_precision)
        features = encode_faces(imgpaths, encoder, enc_batch_size, enc_area)
        if enc_dup_thr and enc_dup_thr != -1:
            features, imgpaths = remove_dupes_overall(features, imgpaths, ('enc', enc_dup_thr, save_dupes, out_dir),
                                                      device=device)
        if group_mode == 'clustering':
            cluster_faces(imgpaths, features, (clusters, clusters_save_all, random_state, group_log, out_dir),
                          device=device)
        if group_mode == 'classification':
            classify_faces(imgpaths, features, encoder, (refs, enc_oth_thr, group_log, out_dir), device=device)
    print('Done')

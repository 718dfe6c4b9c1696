"""ctypes binding of libvtf_hip.so (include/vtf.h).

The library is the only compute path: importing a model class without the built library,
or calling it without a GPU, raises -- there is no CPU fallback in the product.
``torch`` is imported first so that the HIP runtime torch already loaded is the one the
library binds to (same soname, libamdhip64.so.7).
"""
import ctypes
import os

import torch  # noqa: F401  (loads the HIP runtime first)

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('VTF_HIP_LIB', os.path.join(os.path.dirname(_HERE), 'lib', 'libvtf_hip.so'))

VTF_E_CAPACITY = -3
VTF_E_DEGENERATE = -4

_c = ctypes
_p = _c.c_void_p
_i64 = _c.c_int64
_i32 = _c.c_int
_f64 = _c.c_double
_f32 = _c.c_float

# name -> argtypes (restype is int unless listed in _RESTYPE)
SIGNATURES = {
    'vtf_last_error': [],
    'vtf_version': [],
    'vtf_release_stream': [_p],
    'vtf_mtcnn_create': [_p, _i64, _i32, _p],
    'vtf_mtcnn_destroy': [_p],
    'vtf_mtcnn_set_stream': [_p, _p],
    'vtf_mtcnn_detect': [_p, _p, _i32, _i32, _i32, _i32, _i64, _i64, _f64, _p, _p, _p, _i64, _p],
    'vtf_mtcnn_stats': [_p, _p],
    'vtf_mtcnn_stage1_keys': [_p, _i32, _p, _i64, _p],
    'vtf_mtcnn_profile': [_p, _i32, _p, _p, _p, _p],
    'vtf_mtcnn_pnet_level': [_p, _p, _i32, _i32, _i32, _i64, _i64, _i32, _i32, _p, _p],
    'vtf_mtcnn_resample': [_p, _p, _i32, _i32, _i32, _i64, _i64, _i32, _i32, _p],
    'vtf_mtcnn_rnet': [_p, _p, _i64, _p, _p],
    'vtf_mtcnn_onet': [_p, _p, _i64, _p, _p, _p],
    'vtf_batched_nms': [_p, _p, _p, _i64, _f64, _p, _p, _p],
    'vtf_facenet_create': [_p, _i64, _i32, _i32, _p],
    'vtf_facenet_destroy': [_p],
    'vtf_facenet_set_stream': [_p, _p],
    'vtf_facenet_forward': [_p, _p, _i64, _p],
    'vtf_facenet_encode_crops': [_p, _p, _i32, _i32, _i32, _i64, _i64, _p, _i32, _i64, _p],
    'vtf_vit_create': [_p, _i64, _i32, _i32, _i32, _p],
    'vtf_vit_destroy': [_p],
    'vtf_vit_set_stream': [_p, _p],
    'vtf_vit_set_precision': [_p, _i32],
    'vtf_vit_forward': [_p, _p, _i64, _p],
    'vtf_vit_encode_crops': [_p, _p, _i32, _i32, _i32, _i64, _i64, _p, _i32, _i64, _p],
    'vtf_blob_from_crops': [_p, _i32, _i32, _i32, _i64, _i64, _p, _i64, _i32, _f32, _f32, _p, _p],
    'vtf_gemm_split': [_p, _p, _i64, _i32, _i32, _p, _p, _p],
    'vtf_cosine_dedupe': [_p, _i64, _i64, _p, _p, _p],
    'vtf_cosine_dedupe_rows': [_p, _i64, _i64, _i64, _i64, _p, _p, _p],
    'vtf_group_create': [_i32, _p],
    'vtf_group_destroy': [_p],
    'vtf_group_set_stream': [_p, _p],
    'vtf_colstats': [_p, _p, _i64, _i64, _p, _p, _p],
    'vtf_sqdist_rows': [_p, _p, _i64, _i64, _p, _i32, _p],
    'vtf_kmeans_step': [_p, _p, _i64, _i64, _p, _i32, _p, _p, _p, _p],
    'vtf_kmeans_average': [_p, _p, _p, _p, _i32, _i64, _p],
    'vtf_center_dist': [_p, _p, _i64, _i64, _p, _p, _p],
    'vtf_pairwise_euclidean': [_p, _p, _i64, _i64, _p],
    'vtf_silhouette_samples': [_p, _p, _i64, _p, _i32, _p, _p],
    'vtf_silhouette_sweep': [_p, _p, _i64, _i64, _i64, _i64, _p, _i32, _p, _p, _p],
    'vtf_cluster_sums': [_p, _p, _i64, _i64, _p, _i32, _p, _p, _p],
    'vtf_cluster_dist': [_p, _p, _i64, _i64, _p, _i32, _p, _p],
    'vtf_yolo_create': [_p, _i64, _i32, _i32, _p],
    'vtf_yolo_destroy': [_p],
    'vtf_yolo_set_stream': [_p, _p],
    'vtf_yolo_detect': [_p, _p, _i32, _i32, _i32, _i32, _i64, _i64, _p, _p, _p, _i64, _p],
    'vtf_yolo_input_size': [_i32, _i32, _p],
    'vtf_yolo_letterbox': [_p, _p, _i32, _i32, _i32, _i64, _i64, _p],
    'vtf_yolo_net': [_p, _p, _i32, _i32, _i32, _p, _p, _p],
    'vtf_yolo_postprocess': [_p, _p, _p, _p, _i32, _i32, _i32, _p, _p, _p, _i64, _p],
    'vtf_yolo_profile': [_p, _i32, _p, _p, _p, _p],
    'vtf_cosine_classify': [_p, _i64, _p, _i64, _i64, _p, _p, _p],
    'vtf_cosine_distances_xr': [_p, _i64, _p, _i64, _i64, _p, _p],
    'vtf_ahash_crops': [_p, _i32, _i32, _i32, _i64, _i64, _p, _i64, _p, _p],
    'vtf_iom_nms': [_p, _p, _p, _i64, _f32, _p, _p, _p],
    'vtf_boxes_to_crops': [_p, _p, _i32, _i32, _i32, _p, _i32, _p, _p, _p, _i64, _p, _p],
    'vtf_mtcnn_detect_crops': [_p, _p, _i32, _i32, _i32, _i32, _i64, _i64, _f64, _p, _i32, _p, _p, _i64, _p],
    'vtf_yolo_detect_crops': [_p, _p, _i32, _i32, _i32, _i32, _i64, _i64, _p, _i32, _p, _p, _i64, _p],
    'vtf_rcnn_detect_crops': [_p, _p, _i32, _i32, _i32, _i32, _i64, _i64, _p, _i32, _p, _p, _i64, _p],
    'vtf_hamming_dedupe': [_p, _i64, _p, _p, _p],
    'vtf_yuv_to_bgr': [_p, _i64, _i32, _i32, _i32, _i32, _i64, _p, _i64, _i64, _p],
    'vtf_rcnn_create': [_p, _i64, _i32, _i32, _p],
    'vtf_rcnn_destroy': [_p],
    'vtf_rcnn_set_stream': [_p, _p],
    'vtf_rcnn_detect': [_p, _p, _i32, _i32, _i32, _i32, _i64, _i64, _p, _p, _p, _i64, _p],
    'vtf_rcnn_input_size': [_i32, _i32, _p],
    'vtf_rcnn_preprocess': [_p, _p, _i32, _i32, _i32, _i64, _i64, _p],
    'vtf_rcnn_rpn_heads': [_p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _p],
    'vtf_rcnn_proposals': [_p, _p, _i64, _p],
    'vtf_roi_align': [_p, _i32, _i32, _i32, _i32, _p, _i64, _f32, _p, _p],
    'vtf_rcnn_rpn_proposals': [_p, _p, _p, _p, _p, _p, _i32, _i32, _i32, _i32, _i32, _p, _i64, _p],
    'vtf_rcnn_profile': [_p, _i32, _p, _p, _p, _p],
}
_RESTYPE = {'vtf_last_error': _c.c_char_p}

_LIB = None


class BoxParams(ctypes.Structure):
    """vtf_box_params (include/vtf.h): the box filter / adjust settings of video_to_faces
    (det_min_score, det_min_size, det_min_border, det_scale, det_square; main.py:50-51)."""
    _fields_ = [('min_score', _c.c_float), ('min_size', _c.c_double), ('min_border', _c.c_double),
                ('scale', _c.c_double * 4), ('square', _c.c_int32), ('adjust', _c.c_int32)]

    @classmethod
    def make(cls, mscore=0.4, msize=50, mborder=5, scale=(1.5, 1.5, 2.2, 1.2), square=True, adjust=True):
        if isinstance(scale, int):  # adjust_boxes accepts one int for all four (detection.py:221-222)
            scale = (scale,) * 4
        return cls(float(mscore), float(msize), float(mborder or 0), (_c.c_double * 4)(*[float(v) for v in scale]),
                   1 if square else 0, 1 if adjust else 0)


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError('libvtf_hip.so not built (%s): run __graft_entry__.build() or '
                              '`make -C video-to-faces_amd`' % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for name, args in SIGNATURES.items():
            if not hasattr(L, name):  # tests/test_native_abi.py checks every header symbol
                continue
            f = getattr(L, name)
            f.argtypes = args
            f.restype = _RESTYPE.get(name, _c.c_int)
        _LIB = L
    return _LIB


class NativeError(RuntimeError):
    pass


def check(rc):
    if rc != 0:
        msg = lib().vtf_last_error().decode(errors='replace')
        if rc == VTF_E_DEGENERATE:
            # the reference fails here with an IndexError (mtcnn.py:159 -> 216/230)
            raise IndexError(msg)
        raise NativeError('vtf error %d: %s' % (rc, msg))
    return rc


def require_gpu(device):
    if not torch.cuda.is_available():
        raise RuntimeError('video-to-faces_amd runs on MI355X GPUs only: no HIP device is visible')
    dev = torch.device(device) if device is not None else torch.device('cuda:0')
    if dev.type != 'cuda':
        raise RuntimeError('video-to-faces_amd has no CPU path (device=%s)' % dev)
    return dev


def ptr(t):
    return ctypes.c_void_p(t.data_ptr())


def stream_ptr(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def device_of(model, default=None):
    """torch.device a model wrapper (RealMTCNN/RealYOLO/AnimeFRCNN/FaceNet/AnimeVIT or their
    handles) runs on."""
    for obj in (model, getattr(model, 'model', None)):
        d = getattr(obj, 'device', None)
        if d is not None:
            return torch.device(d)
    return require_gpu(default)


def run_detect_crops(call, device, B, cap):
    """Drive a vtf_*_detect_crops entry point: call(d_crops, frame_counts, cap, byref(n)) -> rc.
    Returns (device int32 crops [n,5], host int32 per-frame crop counts [B]).  The capacity bound
    is the detector's row count; on VTF_E_CAPACITY the call is repeated with the reported size."""
    import numpy as np
    counts = np.zeros(B, np.int32)
    n = _c.c_int64(0)
    while True:
        crops = torch.empty((max(int(cap), 1), 5), dtype=torch.int32, device=device)
        rc = call(ptr(crops), counts.ctypes.data, int(cap), _c.byref(n))
        if rc == VTF_E_CAPACITY:
            cap = int(n.value)
            continue
        check(rc)
        return crops[:n.value], counts


def frames_view(imgs, device=None):
    """Frames argument of the detectors: np.ndarray uint8 [B,H,W,3] (any non-negative
    strides with packed pixels), a list of frames, or a uint8 CUDA tensor in HBM.  A CUDA
    tensor must live on `device` (the handle's GPU): a kernel on one GPU cannot read another's
    HBM through a raw pointer.
    Returns (base pointer, on_device, B, H, W, frame_stride, row_stride, owner)."""
    import numpy as np
    import torch
    if isinstance(imgs, torch.Tensor):
        t = imgs
        if t.dtype != torch.uint8 or t.dim() != 4 or t.shape[3] != 3:
            raise ValueError('frames tensor must be uint8 [B,H,W,3]')
        if t.is_cuda and device is not None and t.device != torch.device(device):
            raise ValueError('frames tensor is on %s, the model runs on %s' % (t.device, device))
        if t.stride(3) != 1 or t.stride(2) != 3:
            t = t.contiguous()
        B, H, W = t.shape[:3]
        return _c.c_void_p(t.data_ptr()), int(t.is_cuda), B, H, W, t.stride(0), t.stride(1), t
    x = imgs if isinstance(imgs, np.ndarray) else np.stack(imgs)
    if x.dtype != np.uint8 or x.ndim != 4 or x.shape[3] != 3:
        raise ValueError('frames must be uint8 [B,H,W,3]')
    if x.strides[3] != 1 or x.strides[2] != 3 or x.strides[0] < 0 or x.strides[1] < 0:
        x = np.ascontiguousarray(x)
    B, H, W = x.shape[:3]
    return _c.c_void_p(x.ctypes.data), 0, B, H, W, x.strides[0], x.strides[1], x

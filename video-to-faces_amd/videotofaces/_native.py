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
    'vtf_mtcnn_create': [_p, _i64, _i32, _p],
    'vtf_mtcnn_destroy': [_p],
    'vtf_mtcnn_set_stream': [_p, _p],
    'vtf_mtcnn_detect': [_p, _p, _i32, _i32, _i32, _i32, _i64, _i64, _f64, _p, _p, _p, _i64, _p],
    'vtf_mtcnn_stats': [_p, _p],
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
    'vtf_facenet_encode_crops': [_p, _p, _i32, _i32, _i64, _i64, _p, _i64, _p],
    'vtf_vit_create': [_p, _i64, _i32, _i32, _i32, _p],
    'vtf_vit_destroy': [_p],
    'vtf_vit_set_stream': [_p, _p],
    'vtf_vit_set_precision': [_p, _i32],
    'vtf_vit_forward': [_p, _p, _i64, _p],
    'vtf_vit_encode_crops': [_p, _p, _i32, _i32, _i64, _i64, _p, _i64, _p],
    'vtf_blob_from_crops': [_p, _i32, _i32, _i64, _i64, _p, _i64, _i32, _f32, _f32, _p, _p],
    'vtf_cosine_dedupe': [_p, _i64, _i64, _p, _p, _p],
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
    'vtf_ahash_crops': [_p, _i32, _i32, _i64, _i64, _p, _i64, _p, _p],
    'vtf_hamming_dedupe': [_p, _i64, _p, _p, _p],
    'vtf_rcnn_create': [_p, _i64, _i32, _i32, _p],
    'vtf_rcnn_destroy': [_p],
    'vtf_rcnn_set_stream': [_p, _p],
    'vtf_rcnn_detect': [_p, _p, _i32, _i32, _i32, _i32, _i64, _i64, _p, _p, _p, _i64, _p],
    'vtf_rcnn_input_size': [_i32, _i32, _p],
    'vtf_rcnn_preprocess': [_p, _p, _i32, _i32, _i32, _i64, _i64, _p],
    'vtf_rcnn_rpn_heads': [_p, _p, _i32, _i32, _i32, _p, _p, _p, _p, _p],
    'vtf_rcnn_proposals': [_p, _p, _i64, _p],
    'vtf_roi_align': [_p, _i32, _i32, _i32, _i32, _p, _i64, _f32, _p, _p],
    'vtf_rcnn_profile': [_p, _i32, _p, _p, _p, _p],
}
_RESTYPE = {'vtf_last_error': _c.c_char_p}

_LIB = None


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


def frames_view(imgs):
    """Frames argument of the detectors: np.ndarray uint8 [B,H,W,3] (any non-negative
    strides with packed pixels), a list of frames, or a uint8 CUDA tensor in HBM.
    Returns (base pointer, on_device, B, H, W, frame_stride, row_stride, owner)."""
    import numpy as np
    import torch
    if isinstance(imgs, torch.Tensor):
        t = imgs
        if t.dtype != torch.uint8 or t.dim() != 4 or t.shape[3] != 3:
            raise ValueError('frames tensor must be uint8 [B,H,W,3]')
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

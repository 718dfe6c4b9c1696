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
    'vtf_vit_forward': [_p, _p, _i64, _p],
    'vtf_vit_encode_crops': [_p, _p, _i32, _i32, _i64, _i64, _p, _i64, _p],
    'vtf_blob_from_crops': [_p, _i32, _i32, _i64, _i64, _p, _i64, _i32, _f32, _f32, _p, _p],
    'vtf_cosine_dedupe': [_p, _i64, _i64, _p, _p, _p],
    'vtf_cosine_classify': [_p, _i64, _p, _i64, _i64, _p, _p, _p],
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

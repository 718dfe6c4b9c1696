"""ORACLE — TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline leg).

torchvision.ops.batched_nms restated on top of the C NMS core (nms_oracle.c).
torchvision is absent from this image and unpinned by the reference; this follows the
published Python of torchvision/ops/boxes.py (batched_nms, _batched_nms_vanilla,
_batched_nms_coordinate_trick) that the reference calls at
src/videotofaces/detectors/mtcnn.py:196,205,219 and detectors/operations/post.py:8.
"""
import ctypes
import os
import subprocess

import numpy as np
import torch

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB = None


def _lib():
    global _LIB
    if _LIB is None:
        path = os.path.join(_HERE, '_build', 'liboracle.so')
        if not os.path.exists(path):
            subprocess.check_call(['make', '-s', '-C', _HERE])
        lib = ctypes.CDLL(path)
        lib.ora_nms.restype = ctypes.c_int64
        lib.ora_nms.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int64, ctypes.c_double, ctypes.c_void_p]
        _LIB = lib
    return _LIB


def nms(boxes, scores, thr):
    """torchvision.ops.nms on CPU: keep indices, score-descending (stable ties)."""
    b = np.ascontiguousarray(boxes.detach().cpu().numpy(), dtype=np.float32)
    s = np.ascontiguousarray(scores.detach().cpu().numpy(), dtype=np.float32)
    n = b.shape[0]
    keep = np.empty(max(n, 1), np.int64)
    nk = _lib().ora_nms(b.ctypes.data, s.ctypes.data, n, float(thr), keep.ctypes.data)
    return torch.from_numpy(keep[:nk].copy())


def batched_nms(boxes, scores, idxs, thr):
    """torchvision/ops/boxes.py batched_nms: vanilla per-class loop above 4000 coords (CPU),
    coordinate-offset trick otherwise."""
    if boxes.numel() > 4000:
        keep_mask = torch.zeros_like(scores, dtype=torch.bool)
        for class_id in torch.unique(idxs):
            curr = torch.where(idxs == class_id)[0]
            ck = nms(boxes[curr], scores[curr], thr)
            keep_mask[curr[ck]] = True
        keep_indices = torch.where(keep_mask)[0]
        return keep_indices[scores[keep_indices].sort(descending=True)[1]]
    if boxes.numel() == 0:
        return torch.empty((0,), dtype=torch.int64)
    max_coordinate = boxes.max()
    offsets = idxs.to(boxes) * (max_coordinate + torch.tensor(1).to(boxes))
    boxes_for_nms = boxes + offsets[:, None]
    return nms(boxes_for_nms, scores, thr)

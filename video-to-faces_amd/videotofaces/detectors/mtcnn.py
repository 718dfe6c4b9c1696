"""MTCNN face detector on MI355X (drop-in for src/videotofaces/detectors/mtcnn.py).

``RealMTCNN(device, min_face_size=5)`` keeps the reference constructor and ``__call__``
contract (mtcnn.py:312-326): frames ``np.ndarray uint8 [B,H,W,3]`` BGR (any strides, or a
list of frames, or a CUDA uint8 tensor already in HBM) -> ``list[np.ndarray f32 (n_i,5)]``
of ``x1,y1,x2,y2,score`` per frame, in the reference's order.  The whole forward
(preprocess, pyramid, P/R/O-Net, the four NMS passes) runs in libvtf_hip.so.
"""
import ctypes
import os

import numpy as np
import torch

from .. import _native as nat
from .. import synth


class MTCNN:
    """Handle around vtf_mtcnn_* (the reference's nn.Module MTCNN, mtcnn.py:124-252)."""

    def __init__(self, device=None, params=None):
        self.device = nat.require_gpu(device)
        L = nat.lib()
        if params is None:
            params = synth.make_params('mtcnn')
        flat = np.ascontiguousarray(synth.pack(params), dtype=np.float32)
        h = ctypes.c_void_p()
        nat.check(L.vtf_mtcnn_create(flat.ctypes.data, flat.size, self.device.index or 0, ctypes.byref(h)))
        self._h = h
        self.last_stats = None

    def __del__(self):
        h = getattr(self, '_h', None)
        if h and nat._LIB is not None:
            nat._LIB.vtf_mtcnn_destroy(h)
            self._h = None

    def _bind_stream(self):
        nat.check(nat.lib().vtf_mtcnn_set_stream(self._h, nat.stream_ptr(self.device)))

    def forward(self, imgs, minsize=20, return_landmarks=False):
        L = nat.lib()
        self._bind_stream()
        base, on_dev, B, H, W, fstride, rstride, keep_alive = nat.frames_view(imgs, self.device)
        cap = max(64, 256 * B)
        while True:
            boxes = np.empty((cap, 5), np.float32)
            lms = np.empty((cap, 5, 2), np.float32)
            counts = np.empty(B, np.int32)
            total = ctypes.c_int64(0)
            rc = L.vtf_mtcnn_detect(self._h, base, on_dev, B, H, W, fstride, rstride, float(minsize),
                                    boxes.ctypes.data, lms.ctypes.data, counts.ctypes.data, cap,
                                    ctypes.byref(total))
            if rc == nat.VTF_E_CAPACITY:
                cap = int(total.value)
                continue
            nat.check(rc)
            break
        del keep_alive
        st = np.zeros(8, np.int64)
        nat.check(L.vtf_mtcnn_stats(self._h, st.ctypes.data))
        self.last_stats = st
        res, ldm, k = [], [], 0
        for b in range(B):
            n = int(counts[b])
            res.append(boxes[k:k + n].copy())
            ldm.append(lms[k:k + n].copy())
            k += n
        if return_landmarks:
            return res, ldm
        return res

    __call__ = forward

    def detect_crops(self, imgs, minsize, box_params, frame_offset=0):
        """forward + box post-processing on device (detection.py:131-145 without the host):
        -> (device int32 crops [N,5] = frame_offset + frame, x1, y1, x2, y2; host per-frame counts).
        box_params: _native.BoxParams."""
        L = nat.lib()
        self._bind_stream()
        base, on_dev, B, H, W, fstride, rstride, keep_alive = nat.frames_view(imgs, self.device)
        out = nat.run_detect_crops(
            lambda d, c, cap, n: L.vtf_mtcnn_detect_crops(self._h, base, on_dev, B, H, W, fstride, rstride,
                                                          float(minsize), ctypes.byref(box_params), int(frame_offset),
                                                          d, c, cap, n), self.device, B, 64 * B)
        del keep_alive
        st = np.zeros(8, np.int64)
        nat.check(L.vtf_mtcnn_stats(self._h, st.ctypes.data))
        self.last_stats = st
        return out

    def stage1_keys(self, enable=-1):
        """Parity introspection: enable (1 / 0) recording of the stage-1 candidate set for later
        calls; returns the last call's keys (uint64 level << 32 | (b * ph + y) * pw + x, ascending)."""
        n = ctypes.c_int64(0)
        nat.check(nat.lib().vtf_mtcnn_stage1_keys(self._h, int(enable), None, 0, ctypes.byref(n)))
        out = np.empty(max(1, n.value), np.uint64)
        nat.check(nat.lib().vtf_mtcnn_stage1_keys(self._h, -1, out.ctypes.data, n.value, ctypes.byref(n)))
        return out[:n.value]

    def profile(self, enable):
        """Start (enable=True, resets) or stop kernel timing of the fused pyramid+PNet kernel;
        returns (ms, launches, algorithmic flops, frames) accumulated so far."""
        ms, n, fl, fr = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_int64()
        nat.check(nat.lib().vtf_mtcnn_profile(self._h, int(enable), ctypes.byref(ms), ctypes.byref(n),
                                              ctypes.byref(fl), ctypes.byref(fr)))
        return ms.value, n.value, fl.value, fr.value

    # ---- stage-level entry points (parity tests)
    def pnet_level(self, frames_dev, lh, lw):
        B, H, W = frames_dev.shape[:3]
        ph, pw = (lh - 1) // 2 - 4, (lw - 1) // 2 - 4
        prob = torch.empty((B, ph, pw), dtype=torch.float32, device=self.device)
        reg = torch.empty((B, 4, ph, pw), dtype=torch.float32, device=self.device)
        self._bind_stream()
        nat.check(nat.lib().vtf_mtcnn_pnet_level(self._h, nat.ptr(frames_dev), B, H, W, frames_dev.stride(0),
                                                 frames_dev.stride(1), lh, lw, nat.ptr(prob), nat.ptr(reg)))
        return reg, prob

    def resample(self, frames_dev, lh, lw):
        B, H, W = frames_dev.shape[:3]
        out = torch.empty((B, 3, lh, lw), dtype=torch.float32, device=self.device)
        self._bind_stream()
        nat.check(nat.lib().vtf_mtcnn_resample(self._h, nat.ptr(frames_dev), B, H, W, frames_dev.stride(0),
                                               frames_dev.stride(1), lh, lw, nat.ptr(out)))
        return out

    def rnet(self, x):
        x = x.to(self.device, torch.float32).contiguous()
        n = x.shape[0]
        reg = torch.empty((n, 4), dtype=torch.float32, device=self.device)
        prob = torch.empty((n,), dtype=torch.float32, device=self.device)
        self._bind_stream()
        nat.check(nat.lib().vtf_mtcnn_rnet(self._h, nat.ptr(x), n, nat.ptr(reg), nat.ptr(prob)))
        return reg, prob

    def onet(self, x):
        x = x.to(self.device, torch.float32).contiguous()
        n = x.shape[0]
        reg = torch.empty((n, 4), dtype=torch.float32, device=self.device)
        lm = torch.empty((n, 10), dtype=torch.float32, device=self.device)
        prob = torch.empty((n,), dtype=torch.float32, device=self.device)
        self._bind_stream()
        nat.check(nat.lib().vtf_mtcnn_onet(self._h, nat.ptr(x), n, nat.ptr(reg), nat.ptr(lm), nat.ptr(prob)))
        return reg, lm, prob


class RealMTCNN():
    """Drop-in for RealMTCNN (mtcnn.py:312-326)."""

    def __init__(self, device=None, min_face_size=5, weights=None):
        print('Initializing MTCNN model for live-action face detection')
        params = None
        wf = weights or os.path.join(os.getcwd(), 'weights', 'mtcnn_joined.pt')
        if os.path.isfile(wf):
            params = synth.load_real('mtcnn', wf)
        self.model = MTCNN(device, params)
        self.minsize = min_face_size

    def __call__(self, frames):
        with torch.inference_mode():
            boxes = self.model(frames, self.minsize)
        return boxes

    def detect_crops(self, frames, box_params, frame_offset=0):
        return self.model.detect_crops(frames, self.minsize, box_params, frame_offset)


def nms_iom(boxes, scores, classes, thresh):
    """MTCNN._nms_vectorized(boxes, scores, classes, thresh, 'Min') (mtcnn.py:273-309, chain
    suppression) on device tensors, via vtf_iom_nms -> int64 keep indices."""
    dev = boxes.device
    b = boxes[:, :4].to(torch.float32).contiguous()
    s = scores.to(torch.float32).contiguous()
    c = classes.to(torch.int32).contiguous()
    n = b.shape[0]
    keep = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    nk = ctypes.c_int64(0)
    nat.check(nat.lib().vtf_iom_nms(nat.ptr(b), nat.ptr(s), nat.ptr(c), n, float(thresh), nat.ptr(keep),
                                    ctypes.byref(nk), nat.stream_ptr(dev)))
    return keep[:nk.value]


def batched_nms(boxes, scores, idxs, iou_threshold):
    """torchvision.ops.batched_nms on device tensors, via vtf_batched_nms."""
    dev = boxes.device
    b = boxes.to(torch.float32).contiguous()
    s = scores.to(torch.float32).contiguous()
    i = idxs.to(torch.int64).contiguous()
    n = b.shape[0]
    keep = torch.empty(max(n, 1), dtype=torch.int64, device=dev)
    nk = ctypes.c_int64(0)
    nat.check(nat.lib().vtf_batched_nms(nat.ptr(b), nat.ptr(s), nat.ptr(i), n, float(iou_threshold), nat.ptr(keep),
                                        ctypes.byref(nk), nat.stream_ptr(dev)))
    return keep[:nk.value]

"""Faster R-CNN anime-face detector on MI355X (drop-in for src/videotofaces/detectors/rcnn.py).

``AnimeFRCNN(device)`` keeps the reference constructor and ``__call__`` contract
(rcnn.py:154-177): frames ``np.ndarray uint8 [B,H,W,3]`` BGR (or a list of frames, or a uint8
CUDA tensor already in HBM) -> ``(boxes, scores, classes)``: per frame ``np.ndarray f32 (n,4)``
(x1,y1,x2,y2 in frame pixels), ``f32 (n,)`` and ``int64 (n,)``, at most 100 per frame,
score-descending -- what ``FasterRCNN.forward`` returns, including its short list when the
last frames hold no RPN proposal (rcnn.py:111).  The whole forward (letterbox, ResNet50 + FPN,
RPN top-k/decode/NMS, multi-level RoIAlign, RoI head, per-image NMS, scale_boxes) runs in
libvtf_hip.so.
"""
import ctypes
import os

import numpy as np
import torch

from .. import _native as nat
from .. import synth

STRIDES = (4, 8, 16, 32, 64)


def input_size(H, W):
    """(h, w, Hp, Wp): resize_cv2's keep-ratio size for (800, 1333) and the x32-padded input."""
    o = np.zeros(4, np.int32)
    nat.check(nat.lib().vtf_rcnn_input_size(H, W, o.ctypes.data))
    return tuple(int(v) for v in o)


class FasterRCNN:
    """Handle around vtf_rcnn_* (the reference's nn.Module FasterRCNN, rcnn.py:127-151).
    precision 'fp32' (parity) or 'bf16' (bf16 operands and activations, fp32 accumulation)."""

    def __init__(self, device=None, params=None, precision='fp32'):
        self.device = nat.require_gpu(device)
        if precision not in ('fp32', 'bf16'):
            raise ValueError('precision must be fp32 or bf16')
        self.precision = precision
        if params is None:
            params = synth.make_params('rcnn')
        flat = np.ascontiguousarray(synth.pack(params), dtype=np.float32)
        h = ctypes.c_void_p()
        nat.check(nat.lib().vtf_rcnn_create(flat.ctypes.data, flat.size, self.device.index or 0,
                                            int(precision == 'bf16'), ctypes.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, '_h', None)
        if h and nat._LIB is not None:
            nat._LIB.vtf_rcnn_destroy(h)
            self._h = None

    def _bind_stream(self):
        nat.check(nat.lib().vtf_rcnn_set_stream(self._h, nat.stream_ptr(self.device)))

    def forward(self, imgs):
        L = nat.lib()
        self._bind_stream()
        base, on_dev, B, H, W, fs, rs, keep_alive = nat.frames_view(imgs, self.device)
        cap = max(100, 100 * B)
        boxes = np.empty((cap, 4), np.float32)
        scores = np.empty(cap, np.float32)
        counts = np.empty(B, np.int32)
        total = ctypes.c_int64(0)
        nat.check(L.vtf_rcnn_detect(self._h, base, on_dev, B, H, W, fs, rs, boxes.ctypes.data, scores.ctypes.data,
                                    counts.ctypes.data, cap, ctypes.byref(total)))
        del keep_alive
        bs, ss, cs, k = [], [], [], 0
        for b in range(B):
            n = int(counts[b])
            if n < 0:  # past max(imidx) + 1: absent from the reference's lists (rcnn.py:111)
                break
            bs.append(boxes[k:k + n].copy())
            ss.append(scores[k:k + n].copy())
            cs.append(np.zeros(n, np.int64))
            k += n
        return bs, ss, cs

    __call__ = forward

    def detect_crops(self, imgs, box_params, frame_offset=0):
        """forward + box post-processing on device -> (device int32 crops [N,5], host per-frame
        counts), as MTCNN.detect_crops."""
        L = nat.lib()
        self._bind_stream()
        base, on_dev, B, H, W, fs, rs, keep_alive = nat.frames_view(imgs, self.device)
        out = nat.run_detect_crops(
            lambda d, c, cap, n: L.vtf_rcnn_detect_crops(self._h, base, on_dev, B, H, W, fs, rs,
                                                         ctypes.byref(box_params), int(frame_offset), d, c, cap, n),
            self.device, B, 100 * B)
        del keep_alive
        return out

    def profile(self, enable):
        """Start (enable=True, resets) or stop timing of the body+FPN+RPN conv stack; returns
        (ms, launches, algorithmic flops, frames) accumulated so far."""
        ms, n, fl, fr = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_int64()
        nat.check(nat.lib().vtf_rcnn_profile(self._h, int(enable), ctypes.byref(ms), ctypes.byref(n),
                                             ctypes.byref(fl), ctypes.byref(fr)))
        return ms.value, n.value, fl.value, fr.value

    # ---- stage-level entry points (parity tests)
    def preprocess(self, frames_dev):
        B, H, W = frames_dev.shape[:3]
        _, _, Hp, Wp = input_size(H, W)
        out = torch.empty((B, Hp, Wp, 8), dtype=torch.float32, device=self.device)
        self._bind_stream()
        nat.check(nat.lib().vtf_rcnn_preprocess(self._h, nat.ptr(frames_dev), B, H, W, frames_dev.stride(0),
                                                frames_dev.stride(1), nat.ptr(out)))
        return out

    def rpn_heads(self, x, raw=False):
        """x: NCHW fp32 [B,3,Hp,Wp] -> per level (reg [B,h*w*3,4], log [B,h*w*3,1]) like
        RegionProposalNetwork.head (rcnn.py:42-47); raw=True: the NHWC [B,h,w,15] head maps."""
        x = x.to(self.device, torch.float32).contiguous()
        B, _, Hp, Wp = x.shape
        h, w, heads = Hp // 4, Wp // 4, []
        for _ in STRIDES:
            heads.append(torch.empty((B, h, w, 15), dtype=torch.float32, device=self.device))
            h, w = (h - 1) // 2 + 1, (w - 1) // 2 + 1
        self._bind_stream()
        nat.check(nat.lib().vtf_rcnn_rpn_heads(self._h, nat.ptr(x), B, Hp, Wp, *[nat.ptr(t) for t in heads]))
        if raw:
            return heads
        out = []
        for t in heads:
            t = t.reshape(B, -1, 15)
            log = t[..., :3].reshape(B, -1, 1)
            reg = t[..., 3:].reshape(B, -1, 4)
            out.append((reg, log))
        return out

    def rpn_proposals(self, heads_nhwc, Hp, Wp, h_used, w_used):
        """RPN selection (rcnn.py:49-82) from given head maps (NHWC [B,h,w,15] device tensors, as
        rpn_heads computes them) -> (boxes f32 [n,4], image index int64 [n])."""
        hs = [t.to(self.device, torch.float32).contiguous() for t in heads_nhwc]
        B = hs[0].shape[0]
        L = nat.lib()
        cap = 1000 * B
        n = ctypes.c_int64(0)
        buf = np.empty((cap, 5), np.float32)
        self._bind_stream()
        nat.check(L.vtf_rcnn_rpn_proposals(self._h, *[nat.ptr(t) for t in hs], B, Hp, Wp, h_used, w_used,
                                           buf.ctypes.data, cap, ctypes.byref(n)))
        buf = buf[:n.value]
        return buf[:, 1:].copy(), buf[:, 0].astype(np.int64)

    def proposals(self):
        """RPN proposals of the last call: (boxes f32 [n,4], image index int64 [n])."""
        n = ctypes.c_int64(0)
        L = nat.lib()
        cap = 4096
        while True:
            buf = np.empty((cap, 5), np.float32)
            rc = L.vtf_rcnn_proposals(self._h, buf.ctypes.data, cap, ctypes.byref(n))
            if rc == nat.VTF_E_CAPACITY:
                cap = int(n.value)
                continue
            nat.check(rc)
            break
        buf = buf[:n.value]
        return buf[:, 1:].copy(), buf[:, 0].astype(np.int64)


def roi_align(fmap, rois, spatial_scale):
    """torchvision.ops.roi_align(fmap, rois, (7, 7), spatial_scale, 0, True) on device:
    fmap NCHW [N,C,H,W], rois [R,5] -> [R,C,7,7] (vtf_roi_align)."""
    dev = fmap.device
    f = fmap.to(torch.float32).permute(0, 2, 3, 1).contiguous()
    r = rois.to(dev, torch.float32).contiguous()
    N, H, W, C = f.shape
    R = r.shape[0]
    out = torch.empty((R, 7, 7, C), dtype=torch.float32, device=dev)
    nat.check(nat.lib().vtf_roi_align(nat.ptr(f), N, H, W, C, nat.ptr(r), R, ctypes.c_float(spatial_scale),
                                      nat.ptr(out), nat.stream_ptr(dev)))
    return out.permute(0, 3, 1, 2)


class AnimeFRCNN():
    """Drop-in for AnimeFRCNN (rcnn.py:154-177)."""

    def __init__(self, device=None, weights=None, precision='fp32'):
        print('Initializing FasterRCNN model for anime face detection')
        params = None
        wf = weights or os.path.join(os.getcwd(), 'weights', 'frcnn_anime.pt')
        if os.path.isfile(wf):
            params = synth.load_real('rcnn', wf)
        self.model = FasterRCNN(device, params, precision)

    def __call__(self, imgs):
        with torch.inference_mode():
            return self.model(imgs)

    def detect_crops(self, frames, box_params, frame_offset=0):
        return self.model.detect_crops(frames, box_params, frame_offset)

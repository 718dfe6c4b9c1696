"""YOLOv3 face detector on MI355X (drop-in for src/videotofaces/detectors/yolo.py).

``RealYOLO(device)`` keeps the reference constructor and ``__call__`` contract
(yolo.py:179-191): frames ``np.ndarray uint8 [B,H,W,3]`` BGR (or a list of frames, or a
uint8 CUDA tensor already in HBM) -> ``(boxes, scores, classes)``: per frame
``np.ndarray f32 (n,4)`` (x1,y1,x2,y2 in frame pixels), ``f32 (n,)`` and ``int64 (n,)``,
at most 100 per frame, score-descending -- exactly what ``YOLOv3.forward`` returns.
The whole forward (letterbox, Darknet53/neck/head, decode, per-image NMS, top-100,
scale_boxes) runs in libvtf_hip.so.
"""
import ctypes
import os

import numpy as np
import torch

from .. import _native as nat
from .. import synth


def input_size(H, W):
    """(h, w, Hp, Wp): resize_cv2's keep-ratio size and the x32-padded net input (prep.py:71-92)."""
    o = np.zeros(4, np.int32)
    nat.check(nat.lib().vtf_yolo_input_size(H, W, o.ctypes.data))
    return tuple(int(v) for v in o)


class YOLOv3:
    """Handle around vtf_yolo_* (the reference's nn.Module YOLOv3, yolo.py:123-176).
    precision 'fp32' (parity: fp32 MFMA; 1e-4-level vs the reference), 'x3' (fp32-grade: each fp32
    operand as three bf16 terms, six bf16 MFMAs per product, fp32 exponent range) or 'bf16'
    (bf16 operands and activations, fp32 accumulation)."""

    _MODES = {'fp32': 0, 'bf16': 1, 'x3': 2}

    def __init__(self, device=None, params=None, precision='fp32'):
        self.device = nat.require_gpu(device)
        if precision not in self._MODES:
            raise ValueError('precision must be fp32, x3 or bf16')
        self.precision = precision
        if params is None:
            params = synth.make_params('yolo')
        flat = np.ascontiguousarray(synth.pack(params), dtype=np.float32)
        h = ctypes.c_void_p()
        nat.check(nat.lib().vtf_yolo_create(flat.ctypes.data, flat.size, self.device.index or 0,
                                            self._MODES[precision], ctypes.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, '_h', None)
        if h and nat._LIB is not None:
            nat._LIB.vtf_yolo_destroy(h)
            self._h = None

    def _bind_stream(self):
        nat.check(nat.lib().vtf_yolo_set_stream(self._h, nat.stream_ptr(self.device)))

    @staticmethod
    def _split(B, counts, boxes, scores):
        bs, ss, cs, k = [], [], [], 0
        for b in range(B):
            n = int(counts[b])
            bs.append(boxes[k:k + n].copy())
            ss.append(scores[k:k + n].copy())
            cs.append(np.zeros(n, np.int64))
            k += n
        return bs, ss, cs

    def _run(self, fn, B):
        cap = max(100, 100 * B)
        boxes = np.empty((cap, 4), np.float32)
        scores = np.empty(cap, np.float32)
        counts = np.empty(B, np.int32)
        total = ctypes.c_int64(0)
        nat.check(fn(boxes.ctypes.data, scores.ctypes.data, counts.ctypes.data, cap, ctypes.byref(total)))
        return self._split(B, counts, boxes, scores)

    def forward(self, imgs):
        L = nat.lib()
        self._bind_stream()
        base, on_dev, B, H, W, fs, rs, keep_alive = nat.frames_view(imgs, self.device)
        out = self._run(lambda *o: L.vtf_yolo_detect(self._h, base, on_dev, B, H, W, fs, rs, *o), B)
        del keep_alive
        return out

    __call__ = forward

    def detect_crops(self, imgs, box_params, frame_offset=0):
        """forward + box post-processing on device -> (device int32 crops [N,5], host per-frame
        counts), as MTCNN.detect_crops."""
        L = nat.lib()
        self._bind_stream()
        base, on_dev, B, H, W, fs, rs, keep_alive = nat.frames_view(imgs, self.device)
        out = nat.run_detect_crops(
            lambda d, c, cap, n: L.vtf_yolo_detect_crops(self._h, base, on_dev, B, H, W, fs, rs,
                                                         ctypes.byref(box_params), int(frame_offset), d, c, cap, n),
            self.device, B, 100 * B)
        del keep_alive
        return out

    def profile(self, enable):
        """Start (enable=True, resets) or stop timing of the conv stack (75 conv launches
        per call); returns (ms, launches, algorithmic flops, frames) accumulated so far."""
        ms, n, fl, fr = ctypes.c_double(), ctypes.c_int64(), ctypes.c_double(), ctypes.c_int64()
        nat.check(nat.lib().vtf_yolo_profile(self._h, int(enable), ctypes.byref(ms), ctypes.byref(n),
                                             ctypes.byref(fl), ctypes.byref(fr)))
        return ms.value, n.value, fl.value, fr.value

    # ---- stage-level entry points (parity tests)
    def letterbox(self, frames_dev):
        B, H, W = frames_dev.shape[:3]
        _, _, Hp, Wp = input_size(H, W)
        out = torch.empty((B, Hp, Wp, 8), dtype=torch.float32, device=self.device)
        self._bind_stream()
        nat.check(nat.lib().vtf_yolo_letterbox(self._h, nat.ptr(frames_dev), B, H, W, frames_dev.stride(0),
                                               frames_dev.stride(1), nat.ptr(out)))
        return out

    def net(self, x):
        """x: NCHW fp32 [B,3,Hp,Wp] -> 3 maps NCHW [B,18,h,w] like YOLOv3Head.forward."""
        x = x.to(self.device, torch.float32).contiguous()
        B, _, Hp, Wp = x.shape
        maps = [torch.empty((B, Hp // s, Wp // s, 18), dtype=torch.float32, device=self.device)
                for s in (32, 16, 8)]
        self._bind_stream()
        nat.check(nat.lib().vtf_yolo_net(self._h, nat.ptr(x), B, Hp, Wp, *[nat.ptr(m) for m in maps]))
        return [m.permute(0, 3, 1, 2) for m in maps]

    def postprocess(self, maps, H, W):
        """maps: NCHW [B,18,h,w] (as YOLOv3Head returns) for frames of size HxW."""
        ms = [m.to(self.device, torch.float32).permute(0, 2, 3, 1).contiguous() for m in maps]
        B = ms[0].shape[0]
        self._bind_stream()
        L = nat.lib()
        return self._run(lambda *o: L.vtf_yolo_postprocess(self._h, *[nat.ptr(m) for m in ms], B, H, W, *o), B)


class RealYOLO():
    """Drop-in for RealYOLO (yolo.py:179-191)."""

    def __init__(self, device=None, weights=None, precision='fp32'):
        print('Initializing YOLOv3 model for live-action face detection')
        params = None
        wf = weights or os.path.join(os.getcwd(), 'weights', 'yolov3_wider.pt')
        if os.path.isfile(wf):
            params = synth.load_real('yolo', wf)
        self.model = YOLOv3(device, params, precision)

    def __call__(self, imgs):
        with torch.inference_mode():
            return self.model(imgs)

    def detect_crops(self, frames, box_params, frame_offset=0):
        return self.model.detect_crops(frames, box_params, frame_offset)

"""FaceNet encoder on MI355X (drop-in for src/videotofaces/encoders/facenet.py).

``FaceNet(device, isC=False)`` keeps the reference constructor and ``__call__`` contract
(facenet.py:157-183): ``list[np.ndarray uint8 (h,w,3) BGR]`` -> ``np.ndarray f32 [N,512]``
(L2-normalised), in input order.  The blob step (resize to 160x160, (x-127.5)/128, RGB)
and the whole InceptionResnetV1 run in libvtf_hip.so.
``precision='fp32'`` (default, parity mode) or ``'bf16'`` (bf16 operands, fp32 accumulate).
"""
import ctypes
import os

import numpy as np
import torch

from .. import _native as nat
from .. import synth


class InceptionResnetV1:
    """Handle around vtf_facenet_* (the reference's nn.Module, facenet.py:123-154)."""

    def __init__(self, device=None, params=None, precision='fp32'):
        self.device = nat.require_gpu(device)
        if precision not in ('fp32', 'bf16'):
            raise ValueError('precision must be fp32 or bf16')
        self.precision = precision
        if params is None:
            params = synth.make_params('facenet')
        flat = np.ascontiguousarray(synth.pack(params), dtype=np.float32)
        h = ctypes.c_void_p()
        nat.check(nat.lib().vtf_facenet_create(flat.ctypes.data, flat.size, self.device.index or 0,
                                               1 if precision == 'bf16' else 0, ctypes.byref(h)))
        self._h = h

    def __del__(self):
        h = getattr(self, '_h', None)
        if h and nat._LIB is not None:
            nat._LIB.vtf_facenet_destroy(h)
            self._h = None

    def _bind(self):
        nat.check(nat.lib().vtf_facenet_set_stream(self._h, nat.stream_ptr(self.device)))

    def forward(self, x):
        """x: float tensor [N,3,160,160] (blob) -> [N,512] device tensor."""
        x = x.to(self.device, torch.float32).contiguous()
        n = x.shape[0]
        out = torch.empty((n, 512), dtype=torch.float32, device=self.device)
        self._bind()
        nat.check(nat.lib().vtf_facenet_forward(self._h, nat.ptr(x), n, nat.ptr(out)))
        return out

    __call__ = forward

    def encode_crops(self, frames_dev, crops):
        """frames_dev: CUDA uint8 [F,H,W,3]; crops int [N,5] (frame, x1, y1, x2, y2): a host array
        (validated against the frames) or a CUDA int32 tensor on this device (e.g. from
        detect_crops) -> [N,D] embeddings on device."""
        if isinstance(crops, torch.Tensor) and crops.is_cuda:
            if crops.device != self.device:
                raise ValueError('crops are on %s, the encoder runs on %s' % (crops.device, self.device))
            c = crops.to(torch.int32).contiguous().reshape(-1, 5)
            on_dev, cptr = 1, nat.ptr(c)
        else:
            c = np.ascontiguousarray(crops, dtype=np.int32).reshape(-1, 5)
            on_dev, cptr = 0, c.ctypes.data
        n = c.shape[0]
        out = torch.empty((n, 512), dtype=torch.float32, device=self.device)
        if n == 0:
            return out
        if frames_dev.device != self.device:
            raise ValueError('frames are on %s, the encoder runs on %s' % (frames_dev.device, self.device))
        F, H, W = frames_dev.shape[:3]
        self._bind()
        nat.check(nat.lib().vtf_facenet_encode_crops(self._h, nat.ptr(frames_dev), F, H, W, frames_dev.stride(0),
                                    frames_dev.stride(1), cptr, on_dev, n, nat.ptr(out)))
        return out


def blob_from_images(images, size, mean, scale, device):
    """cv2.dnn.blobFromImages(images, scale, (size,size), (mean,)*3, swapRB=True) on device:
    list of uint8 BGR crops -> fp32 [N,3,size,size]."""
    n = len(images)
    out = torch.empty((n, 3, size, size), dtype=torch.float32, device=device)
    if n == 0:
        return out
    # pack the crops as 1-row-frame strips of one upload: each crop becomes its own frame
    Hm = max(im.shape[0] for im in images)
    Wm = max(im.shape[1] for im in images)
    buf = np.zeros((n, Hm, Wm, 3), np.uint8)
    crops = np.zeros((n, 5), np.int32)
    for i, im in enumerate(images):
        h, w = im.shape[:2]
        buf[i, :h, :w] = im
        crops[i] = (i, 0, 0, w, h)
    fr = torch.from_numpy(buf).to(device)
    dc = torch.from_numpy(crops).to(device)
    nat.check(nat.lib().vtf_blob_from_crops(nat.ptr(fr), n, Hm, Wm, fr.stride(0), fr.stride(1), nat.ptr(dc), n, size,
                                            ctypes.c_float(mean), ctypes.c_float(scale), nat.ptr(out),
                                            nat.stream_ptr(device)))
    return out


class FaceNet():
    """Drop-in for FaceNet (facenet.py:157-183)."""

    stor = 'https://github.com/timesler/facenet-pytorch/releases/download/v2.2.9/'
    links = {'vgg': stor + '20180402-114759-vggface2.pt', 'casia': stor + '20180408-102900-casia-webface.pt'}

    def __init__(self, device=None, isC=False, precision='fp32', weights=None):
        src = 'vgg' if not isC else 'casia'
        print('Initializing FaceNet %s model for live-action face encoding' % src.upper())
        params = None
        wf = weights or os.path.join(os.getcwd(), 'weights', 'facenet_' + src + '.pt')
        if os.path.isfile(wf):
            params = synth.load_real('facenet', wf)
        self.model = InceptionResnetV1(device, params, precision)

    def __call__(self, images):
        inp = blob_from_images(images, 160, 127.5, 1 / 128, self.model.device)
        with torch.inference_mode():
            out = self.model(inp)
        return out.cpu().numpy()

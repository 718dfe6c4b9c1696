"""ViT anime-face encoder on MI355X (drop-in for src/videotofaces/encoders/vit.py).

``AnimeVIT(device, isL=False)`` keeps the reference constructor and ``__call__`` contract
(vit.py:105-146): ``list[np.ndarray uint8 (h,w,3) BGR]`` -> ``np.ndarray f32 [N,768|1024]``
(LayerNorm of the CLS token, not L2-normalised).  Blob (128x128, (x-127.5)/127.5, RGB) and
the whole ViT-B/16 or ViT-L/16 run in libvtf_hip.so: fp32 operands, GEMMs on the fp16 matrix
cores with split operands (fp32-grade products; guarded, fp32 MFMA fallback) or on fp32 MFMA.
"""
import ctypes
import os

import numpy as np
import torch

from .. import _native as nat
from .. import synth
from .facenet import blob_from_images


class ViT:
    """Handle around vtf_vit_* (the reference's nn.Module ViT, vit.py:80-102)."""

    def __init__(self, device=None, params=None, isL=False, precision='f16x'):
        """precision: 'fp32' (fp32 MFMA) or 'f16x' (fp32-grade split-fp16 MFMA products, guarded:
        an out-of-range operand re-runs the forward in fp32)."""
        if precision not in ('fp32', 'f16x'):
            raise ValueError("precision must be 'fp32' or 'f16x'")
        self.device = nat.require_gpu(device)
        self.name = 'vit_l' if isL else 'vit_b'
        self.dim, depth = (1024, 24) if isL else (768, 12)
        if params is None:
            params = synth.make_params(self.name)
        flat = np.ascontiguousarray(synth.pack(params), dtype=np.float32)
        h = ctypes.c_void_p()
        nat.check(nat.lib().vtf_vit_create(flat.ctypes.data, flat.size, self.dim, depth, self.device.index or 0,
                                           ctypes.byref(h)))
        self._h = h
        self.precision = precision
        nat.check(nat.lib().vtf_vit_set_precision(h, 2 if precision == 'f16x' else 0))

    def __del__(self):
        h = getattr(self, '_h', None)
        if h and nat._LIB is not None:
            nat._LIB.vtf_vit_destroy(h)
            self._h = None

    def _bind(self):
        nat.check(nat.lib().vtf_vit_set_stream(self._h, nat.stream_ptr(self.device)))

    def forward(self, x):
        x = x.to(self.device, torch.float32).contiguous()
        n = x.shape[0]
        out = torch.empty((n, self.dim), dtype=torch.float32, device=self.device)
        self._bind()
        nat.check(nat.lib().vtf_vit_forward(self._h, nat.ptr(x), n, nat.ptr(out)))
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
        out = torch.empty((n, self.dim), dtype=torch.float32, device=self.device)
        if n == 0:
            return out
        if frames_dev.device != self.device:
            raise ValueError('frames are on %s, the encoder runs on %s' % (frames_dev.device, self.device))
        F, H, W = frames_dev.shape[:3]
        self._bind()
        nat.check(nat.lib().vtf_vit_encode_crops(self._h, nat.ptr(frames_dev), F, H, W, frames_dev.stride(0),
                                    frames_dev.stride(1), cptr, on_dev, n, nat.ptr(out)))
        return out


class AnimeVIT():
    """Drop-in for AnimeVIT (vit.py:105-146)."""

    links = {'B16': '1hEtmrzlh7RrXuUoxi5eqMQd5yIirQ-XC', 'L16': '1eZai1_gjos6TNeQZg6IY-cIWxtg0Pxah'}

    def __init__(self, device=None, isL=False, weights=None, precision='fp32'):
        """precision: 'fp32' (default: fp32 MFMA, the parity mode) or 'f16x' (guarded split-fp16
        GEMMs, fp32-grade products, ~1.7x faster; 'bf16' is read as 'f16x')."""
        src = 'B16' if not isL else 'L16'
        print('Initializing ViT %s model for anime face encoding' % src)
        params = None
        wf = weights or os.path.join(os.getcwd(), 'weights', 'vit_anime_' + src.lower() + '.pt')
        if os.path.isfile(wf):
            params = synth.load_real('vit_l' if isL else 'vit_b', wf)
        self.model = ViT(device, params, isL, precision='f16x' if precision in ('f16x', 'bf16') else 'fp32')

    def __call__(self, images):
        inp = blob_from_images(images, 128, 127.5, 1 / 127.5, self.model.device)
        with torch.inference_mode():
            out = self.model(inp)
        return out.cpu().numpy()

"""Video frame source for process_video (src/videotofaces/detection.py:68-111) on raw YUV streams.

The reference decodes with cv2.VideoCapture (seek or grab/retrieve, detection.py:98-111) or
decord (get_batch, :95-97) and hands the detector uint8 BGR frames.  This image has no codec
(cv2, decord, FFmpeg, rocDecode are all absent), so the container read here is YUV4MPEG2 -- the
uncompressed stream any decoder emits (`ffmpeg -i in.mp4 -f yuv4mpegpipe out.y4m`): the file is
memory-mapped, the sampled frames' planes are gathered into pinned host memory as they lie in
the file (1.5 bytes per 4:2:0 pixel over PCIe, not 3) and one launch of vtf_yuv_to_bgr turns
them into the BGR frames in HBM that the detectors read in place.

YUV4MPEG2: a header line 'YUV4MPEG2 W<w> H<h> F<num>:<den> [I..] [A..] [C<chroma>] [X..]\\n',
then per frame 'FRAME[ params]\\n' + Y [H][W] + U, V planes (4:2:0: ceil(W/2) x ceil(H/2)).
"""
import mmap
import os

import numpy as np

_CHROMA = {'420jpeg': 420, '420paldv': 420, '420mpeg2': 420, '420': 420, '422': 422, '444': 444, 'mono': 400}


def frame_bytes(H, W, chroma=420):
    """bytes of one frame's planes: Y [H][W] + U, V of the chroma size (none for mono)."""
    if chroma == 400:
        return H * W
    sx, sy = (0 if chroma == 444 else 1), (1 if chroma == 420 else 0)
    return H * W + 2 * ((W + sx) >> sx) * ((H + sy) >> sy)


def write_y4m(path, planes, H, W, fps='30:1', chroma=420, frame_params=None, extra=''):
    """A YUV4MPEG2 file of uint8 planes [F, frame_bytes] (the layout Y4MReader reads);
    frame_params: per-frame header suffixes (or None), extra: more header tags."""
    ctag = {420: 'C420jpeg', 422: 'C422', 444: 'C444', 400: 'Cmono'}[chroma]
    p = np.asarray(planes, np.uint8).reshape(-1, frame_bytes(H, W, chroma))
    with open(path, 'wb') as f:
        f.write(('YUV4MPEG2 W%d H%d F%s Ip A1:1 %s%s\n' % (W, H, fps, ctag, extra)).encode())
        for i, fr in enumerate(p):
            f.write(b'FRAME' + ((' ' + frame_params[i]).encode() if frame_params and frame_params[i] else b'') + b'\n')
            f.write(fr.tobytes())


class Y4MReader:
    """A YUV4MPEG2 file: .n_frames, .fps (rounded as detection.py:84 rounds CAP_PROP_FPS),
    .height, .width, read(indices, device) -> uint8 CUDA tensor [B,H,W,3] BGR."""

    def __init__(self, path):
        self.path = path
        self._f = open(path, 'rb')
        size = os.fstat(self._f.fileno()).st_size
        if size == 0:
            raise ValueError('%s: empty file' % path)
        self._mm = mmap.mmap(self._f.fileno(), 0, access=mmap.ACCESS_READ)
        end = self._mm.find(b'\n')
        if end < 0 or not self._mm[:10] == b'YUV4MPEG2 ':
            raise ValueError('%s: not a YUV4MPEG2 stream' % path)
        hdr = self._mm[10:end].decode('ascii', 'replace').split()
        fields = {}
        for tok in hdr:
            if tok:
                fields.setdefault(tok[0], []).append(tok[1:])
        if 'W' not in fields or 'H' not in fields:
            raise ValueError('%s: header without W / H' % path)
        self.width, self.height = int(fields['W'][0]), int(fields['H'][0])
        num, den = (fields.get('F', ['25:1'])[0].split(':') + ['1'])[:2]
        self.fps_exact = int(num) / max(int(den), 1)
        self.fps = round(self.fps_exact)
        ctag = fields.get('C', ['420jpeg'])[0]
        if ctag not in _CHROMA:
            raise ValueError('%s: chroma C%s not supported (8-bit 420 / 422 / 444 / mono only)' % (path, ctag))
        self.chroma = _CHROMA[ctag]
        self.full_range = any(x.upper() == 'COLORRANGE=FULL' for x in fields.get('X', []))
        self.frame_bytes = frame_bytes(self.height, self.width, self.chroma)
        # frame payload offsets (FRAME headers may carry parameters: walk them)
        offs, p = [], end + 1
        while p < size:
            if self._mm[p:p + 5] != b'FRAME':
                raise ValueError('%s: bad frame header at byte %d' % (path, p))
            e = self._mm.find(b'\n', p)
            if e < 0 or e + 1 + self.frame_bytes > size:
                break  # a truncated last frame is not a frame (VideoCapture stops there too)
            offs.append(e + 1)
            p = e + 1 + self.frame_bytes
        self.offsets = np.asarray(offs, np.int64)
        self.n_frames = len(offs)
        self._pinned = None

    def close(self):
        if self._mm is not None:
            self._mm.close()
            self._f.close()
            self._mm = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def planes(self, indices):
        """host uint8 [B, frame_bytes]: the raw planes of the given frames (a copy)."""
        idx = np.asarray(indices, np.int64).reshape(-1)
        if idx.size and (idx.min() < 0 or idx.max() >= self.n_frames):
            raise IndexError('frame index out of range [0, %d)' % self.n_frames)
        out = np.empty((idx.size, self.frame_bytes), np.uint8)
        for k, i in enumerate(idx.tolist()):
            o = int(self.offsets[i])
            out[k] = np.frombuffer(self._mm, np.uint8, self.frame_bytes, o)
        return out

    def read(self, indices, device=None):
        """BGR frames [B,H,W,3] uint8 in HBM of `device` (default cuda:0): the planes are gathered
        into a pinned staging buffer, copied with one async H2D and converted by vtf_yuv_to_bgr."""
        import torch
        from . import _native as nat
        dev = nat.require_gpu(device)
        idx = np.asarray(indices, np.int64).reshape(-1)
        B, FB = idx.size, self.frame_bytes
        out = torch.empty((B, self.height, self.width, 3), dtype=torch.uint8, device=dev)
        if B == 0:
            return out
        if self._pinned is None or self._pinned.numel() < B * FB:
            self._pinned = torch.empty(B * FB, dtype=torch.uint8, pin_memory=True)
        host = self._pinned[:B * FB].numpy().reshape(B, FB)
        if idx.min() < 0 or idx.max() >= self.n_frames:
            raise IndexError('frame index out of range [0, %d)' % self.n_frames)
        for k, i in enumerate(idx.tolist()):
            host[k] = np.frombuffer(self._mm, np.uint8, FB, int(self.offsets[i]))
        with torch.cuda.device(dev):
            d_yuv = self._pinned[:B * FB].to(dev, non_blocking=True)
            nat.check(nat.lib().vtf_yuv_to_bgr(nat.ptr(d_yuv), B, self.height, self.width, self.chroma,
                                               int(self.full_range), FB, nat.ptr(out), out.stride(0), out.stride(1),
                                               nat.stream_ptr(dev)))
            # the staging buffer is reused by the next read: wait for this copy
            torch.cuda.current_stream(dev).synchronize()
        return out


def yuv_to_bgr(planes, height, width, chroma=420, full_range=False, device=None):
    """uint8 planes [B, frame_bytes] (host array or CUDA tensor) -> BGR CUDA tensor [B,H,W,3]."""
    import torch
    from . import _native as nat
    dev = nat.require_gpu(device)
    t = planes if isinstance(planes, torch.Tensor) else torch.from_numpy(np.ascontiguousarray(planes))
    t = t.to(dev).contiguous()
    if t.dim() == 1:
        t = t[None]
    out = torch.empty((t.shape[0], height, width, 3), dtype=torch.uint8, device=dev)
    nat.check(nat.lib().vtf_yuv_to_bgr(nat.ptr(t), t.shape[0], height, width, chroma, int(bool(full_range)),
                                       t.stride(0), nat.ptr(out), out.stride(0), out.stride(1), nat.stream_ptr(dev)))
    return out

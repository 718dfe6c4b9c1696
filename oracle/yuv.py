"""ORACLE — TEST INFRASTRUCTURE ONLY (tests/).

The frame-source side of process_video (src/videotofaces/detection.py:68-111): the reference's
cv2.VideoCapture / decord return uint8 BGR frames; here decoded frames arrive as planar YUV (a
YUV4MPEG2 stream) and vtf_yuv_to_bgr (csrc/video.hip) converts them on the GPU.  This module
restates that conversion in numpy integer arithmetic (and process_video's frame sampling), so
the GPU path is checked bit for bit against it:
  * BT.601 limited range with OpenCV's fixed-point constants (ITUR_BT_601_CY 1220542, CVR
    1673527, CVG -852492, CUG -409993, CUB 2116026, shift 20, the cvtColor(COLOR_YUV2BGR_I420)
    transform), or full range (1470104, -748826, -360853, 1858077); chroma nearest.
PARITY UNPINNED against the reference's own decoder: cv2 / FFmpeg / decord are not installed
in this image (which colour transform VideoCapture applies is swscale's, not checked here).
"""
import numpy as np

_CH = {420: (1, 1), 422: (1, 0), 444: (0, 0)}


def chroma_size(H, W, chroma):
    if chroma == 400:
        return 0, 0
    sx, sy = _CH[chroma]
    return (H + sy) >> sy, (W + sx) >> sx


def frame_bytes(H, W, chroma):
    ch, cw = chroma_size(H, W, chroma)
    return H * W + 2 * ch * cw


def yuv_to_bgr(planes, H, W, chroma=420, full_range=False):
    """uint8 [B, frame_bytes] -> uint8 [B, H, W, 3] BGR (the transform of csrc/video.hip)."""
    p = np.asarray(planes, np.uint8).reshape(-1, frame_bytes(H, W, chroma))
    B = p.shape[0]
    Y = p[:, :H * W].reshape(B, H, W).astype(np.int64)
    if chroma == 400:
        U = V = np.full((B, H, W), 128, np.int64)
    else:
        ch, cw = chroma_size(H, W, chroma)
        sx, sy = _CH[chroma]
        Up = p[:, H * W:H * W + ch * cw].reshape(B, ch, cw).astype(np.int64)
        Vp = p[:, H * W + ch * cw:].reshape(B, ch, cw).astype(np.int64)
        ys, xs = np.arange(H) >> sy, np.arange(W) >> sx
        U, V = Up[:, ys][:, :, xs], Vp[:, ys][:, :, xs]
    u, v = U - 128, V - 128
    if full_range:
        y = (Y << 20) + (1 << 19)
        r, g, b = y + 1470104 * v, y - 748826 * v - 360853 * u, y + 1858077 * u
    else:
        y = np.maximum(0, Y - 16) * 1220542 + (1 << 19)
        r, g, b = y + 1673527 * v, y - 852492 * v - 409993 * u, y + 2116026 * u
    out = np.stack([b, g, r], -1) >> 20
    return np.clip(out, 0, 255).astype(np.uint8)


def sample_indices(n_frames, fps, video_step, video_fragment=None):
    """process_video's frame sampling (detection.py:85-91)."""
    step = round(fps * video_step)
    bgn = step if not video_fragment or video_fragment[0] < 0 else max(step, round(60 * video_fragment[0] * fps))
    end = n_frames if not video_fragment or video_fragment[1] < 0 else min(n_frames, round(60 * video_fragment[1] * fps + 1))
    return list(range(bgn, end, step))

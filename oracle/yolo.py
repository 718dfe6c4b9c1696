"""ORACLE — TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline leg).

CPU restatement of the reference YOLOv3 face detector (src/videotofaces/detectors/yolo.py,
detectors/operations/{prep,anchor,bbox,post}.py) with torch-CPU functional ops.  The cv2
letterbox resize (prep.py:77) uses oracle.facenet.resize_linear_u8 (cv2 absent: parity-
unpinned step); everything after the resized tensor is pinned by tests/golden/yolo.npz.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from . import nms as onms
from .facenet import resize_linear_u8

BASES = [(32, [(116, 90), (156, 198), (373, 326)]), (16, [(30, 61), (62, 45), (59, 119)]),
         (8, [(10, 13), (16, 30), (33, 23)])]  # yolo.py:125-129


def _cu(P, x, pre, k, s=1):
    """conv_unit: Conv(no bias, pad (k-1)//2) -> BN(eps 1e-5) -> LeakyReLU(0.1) (yolo.py:17-18)"""
    x = F.conv2d(x, P[pre + '.conv.weight'], None, s, (k - 1) // 2)
    x = F.batch_norm(x, P[pre + '.bn.running_mean'], P[pre + '.bn.running_var'], P[pre + '.bn.weight'],
                     P[pre + '.bn.bias'], False, 0.0, 1e-5)
    return F.leaky_relu(x, 0.1, inplace=True)  # nn.LeakyReLU(inplace=True) (basic.py:33)


def _det_block(P, x, pre):
    for i, k in enumerate((1, 3, 1, 3, 1)):
        x = _cu(P, x, '%s.layers.%d' % (pre, i), k)
    return x


def net(params, x):
    """backbone + neck + head (yolo.py:34-120, 139-146) -> 3 maps [B,18,h,w] (stride 32,16,8)."""
    P = {k: torch.from_numpy(np.asarray(v)) for k, v in params.items()}
    with torch.inference_mode():
        x = _cu(P, x, 'backbone.conv1', 3)
        outs = []
        for i, n in enumerate([1, 2, 8, 8, 4]):
            pre = 'backbone.conv_res_block%d' % (i + 1)
            x = _cu(P, x, pre + '.conv', 3, 2)
            for j in range(n):
                y = _cu(P, x, '%s.res%d.conv1' % (pre, j), 1)
                y = _cu(P, y, '%s.res%d.conv2' % (pre, j), 3)
                x = y + x
            outs.append(x)
        x1, x2, x3 = outs[2], outs[3], outs[4]
        y3 = _det_block(P, x3, 'neck.detect1')
        t = F.interpolate(_cu(P, y3, 'neck.conv1', 1), scale_factor=2)
        y2 = _det_block(P, torch.cat((t, x2), 1), 'neck.detect2')
        t = F.interpolate(_cu(P, y2, 'neck.conv2', 1), scale_factor=2)
        y1 = _det_block(P, torch.cat((t, x1), 1), 'neck.detect3')
        maps = []
        for i, y in enumerate((y3, y2, y1)):
            y = _cu(P, y, 'head.convs_bridge.%d' % i, 3)
            maps.append(F.conv2d(y, P['head.convs_pred.%d.weight' % i], P['head.convs_pred.%d.bias' % i]))
        return maps


def preprocess(frames, size=608):
    """prep.py:12-92 with resize_with='cv2', means=None, stdvs=255: keep-ratio resize,
    RGB, /255, zero-pad to a multiple of 32.  Returns x, sz_orig, sz_used."""
    ts, so, su = [], [], []
    for img in frames:
        sz = img.shape[:2]
        scl = min(size / min(sz), size / max(sz))
        n = int(sz[0] * scl + 0.5), int(sz[1] * scl + 0.5)
        im = resize_linear_u8_hw(img, n)
        t = torch.from_numpy(np.ascontiguousarray(im)).to(torch.float32)
        t = t[:, :, [2, 1, 0]]
        t /= torch.tensor(255)
        ts.append(t.permute(2, 0, 1))
        so.append(sz)
        su.append(n)
    hmax = int(math.ceil(max(t.shape[1] for t in ts) / 32) * 32)
    wmax = int(math.ceil(max(t.shape[2] for t in ts) / 32) * 32)
    x = torch.zeros((len(ts), 3, hmax, wmax), dtype=torch.float32)
    for i, t in enumerate(ts):
        x[i, :, :t.shape[1], :t.shape[2]].copy_(t)
    return x, so, su


def resize_linear_u8_hw(img, hw):
    """resize_linear_u8 generalised to a (h, w) target."""
    from .facenet import _coefs
    h, w = img.shape[:2]
    H, W = hw
    if (h, w) == (H, W):
        return img.copy()
    sx0, sx1, a0, a1, ex = _coefs(w, W)
    sy0, sy1, b0, b1, _ = _coefs(h, H)
    src = img.astype(np.int64)

    def hrow(rows):
        r = src[rows]
        v = r[:, sx0] * a0[None, :, None] + r[:, sx1] * a1[None, :, None]
        v[:, ex] = r[:, sx0[ex]] * 2048
        return v
    h0, h1 = hrow(sy0), hrow(sy1)
    t = (((h0 >> 4) * b0[:, None, None]) >> 16) + (((h1 >> 4) * b1[:, None, None]) >> 16)
    return np.clip((t + 2) >> 2, 0, 255).astype(np.uint8)


def priors(hw):
    """get_priors(..., 'center') (anchor.py:20-64)."""
    h, w = hw
    p = []
    for stride, anchors in BASES:
        nx, ny = math.ceil(w / stride), math.ceil(h / stride)
        xs = torch.arange(nx, dtype=torch.float32) * stride + stride / 2
        ys = torch.arange(ny, dtype=torch.float32) * stride + stride / 2
        c = torch.dstack(torch.meshgrid(xs, ys, indexing='xy')).reshape(-1, 2)
        c = c.repeat_interleave(len(anchors), dim=0)
        s = torch.tensor(anchors, dtype=torch.float32).repeat(nx * ny, 1)
        p.append(torch.hstack([c, s]))
    return torch.cat(p)


def postprocess(maps, pri, num_classes=1):
    """YOLOv3.postprocess (yolo.py:151-176) + final_nms (post.py:4-10)."""
    maps = [m.permute(0, 2, 3, 1).reshape(m.shape[0], -1, num_classes + 5) for m in maps]
    map_sizes = [m.shape[1] for m in maps]
    maps = torch.cat(maps, dim=1)
    reg = maps[..., :4]
    obj = maps[..., 4].sigmoid()
    scr = maps[..., 5:].sigmoid()
    n, dim, nc = scr.shape
    reg, scr, obj = reg.reshape(-1, 4), scr.reshape(-1, nc), obj.flatten()
    oidx = torch.nonzero(obj >= 0.005).squeeze(1)
    scr, obj = scr[oidx], obj[oidx]
    s = scr.flatten()
    fidx = torch.nonzero(s > 0.05).squeeze(1)
    idx = torch.div(fidx, nc, rounding_mode='floor')
    s = s[fidx] * obj[idx]
    c = fidx % nc
    idx = oidx[idx]
    imidx = idx.div(dim, rounding_mode='floor')
    strides = [b[0] for b in BASES]
    lvidx = torch.bucketize(idx % dim, torch.tensor(map_sizes).cumsum(0), right=True)
    stidx = torch.tensor(strides)[lvidx].unsqueeze(-1)
    pr = pri[idx % dim]
    xys = stidx * (reg[idx][..., :2].sigmoid() - 0.5) + pr[..., :2]
    whs = pr[..., 2:] * torch.exp(reg[idx][..., 2:])
    boxes = torch.cat([xys - whs / 2, xys + whs / 2], dim=-1)
    res = []
    for i in range(n):
        m = imidx == i
        bi, si, ci = boxes[m], s[m], c[m]
        keep = onms.batched_nms(bi, si, ci, 0.45)[:100]
        res.append((bi[keep], si[keep], ci[keep]))
    return [list(t) for t in zip(*res)] if res else ([], [], [])


def forward(params, frames):
    """YOLOv3.forward (yolo.py:139-149): -> (boxes list, scores list, classes list)."""
    x, so, su = preprocess(frames)
    maps = net(params, x)
    with torch.inference_mode():
        b, s, c = postprocess(maps, priors(x.shape[-2:]))
        scales = torch.tensor(so) / torch.tensor(su)
        scales = scales.flip(1).repeat(1, 2)
        b = [b[i] * scales[i] for i in range(len(b))]
    return [t.numpy() for t in b], [t.numpy() for t in s], [t.numpy() for t in c]

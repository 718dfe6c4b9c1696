"""ORACLE — TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline leg).

CPU restatement of the reference Faster R-CNN anime-face detector
(src/videotofaces/detectors/rcnn.py:16-177, backbones/resnet.py:11-54,
detectors/operations/{prep,anchor,bbox,post,roi}.py) with torch-CPU functional ops.

Third-party pieces the reference reaches through torchvision (absent here, unpinned by the
reference's requirements.txt): ``batched_nms`` (oracle.nms) and ``roi_align`` -- restated
below from torchvision's published CPU kernel (csrc/ops/cpu/roi_align_kernel.cpp:
pre_calc_for_bilinear_interpolate + roi_align_forward_kernel_impl, sampling_ratio 0 =
adaptive grid, aligned=True half-pixel offset).  The cv2 resize of prep.py:77 uses the
INTER_LINEAR restatement (oracle.yolo.resize_linear_u8_hw; parity-unpinned step).
Everything after the resized uint8 image is pinned by tests/golden/rcnn.npz, generated from
the reference's own modules.
"""
import math

import numpy as np
import torch
import torch.nn.functional as F

from . import nms as onms
from .yolo import resize_linear_u8_hw

STRIDES = [4, 8, 16, 32, 64]          # rcnn.py:133
MEANS = [123.675, 116.28, 103.53]     # prep.py:29
STDVS = [58.395, 57.12, 57.375]       # prep.py:30


def anchors():
    """make_anchors([32, 64, 128, 256, 512], [1], [2, 1, 0.5]) (anchor.py:6-17, rcnn.py:134)."""
    mult = [math.sqrt(ar) for ar in [2, 1, 0.5]]
    return [[(d * m, d / m) for m in mult] for d in [32, 64, 128, 256, 512]]


def used_size(H, W):
    """resize_cv2 keep-ratio size for resize=(800, 1333) (prep.py:71-74)."""
    scl = min(800 / min(H, W), 1333 / max(H, W))
    return int(H * scl + 0.5), int(W * scl + 0.5)


def preprocess(frames):
    """preprocess(imgs, dv, (800, 1333), 'cv2') (prep.py:12-92): keep-ratio resize, RGB,
    (x - mean) / std, zero pad to a multiple of 32."""
    ts, so, su = [], [], []
    for img in frames:
        sz = img.shape[:2]
        n = used_size(*sz)
        im = resize_linear_u8_hw(img, n)
        t = torch.from_numpy(np.ascontiguousarray(im)).to(torch.float32)[:, :, [2, 1, 0]]
        t -= torch.tensor(MEANS)
        t /= torch.tensor(STDVS)
        ts.append(t.permute(2, 0, 1))
        so.append(sz)
        su.append(n)
    hmax = int(math.ceil(max(t.shape[1] for t in ts) / 32) * 32)
    wmax = int(math.ceil(max(t.shape[2] for t in ts) / 32) * 32)
    x = torch.zeros((len(ts), 3, hmax, wmax), dtype=torch.float32)
    for i, t in enumerate(ts):
        x[i, :, :t.shape[1], :t.shape[2]].copy_(t)
    return x, so, su


def _cu(P, x, pre, s=1, p=0, relu=True, add=None):
    """ConvUnit(bn=1e-5) (basic.py:37-45): conv (no bias) -> BN -> (+add) -> ReLU."""
    x = F.conv2d(x, P[pre + '.conv.weight'], None, s, p)
    x = F.batch_norm(x, P[pre + '.bn.running_mean'], P[pre + '.bn.running_var'], P[pre + '.bn.weight'],
                     P[pre + '.bn.bias'], False, 0.0, 1e-5)
    if add is not None:
        x = x + add
    return F.relu(x) if relu else x


def body(P, x):
    """ResNet50 (resnet.py:31-54), returns C2..C5."""
    x = _cu(P, x, 'body.layers.0.0', 2, 3)
    x = F.max_pool2d(x, 3, 2, 1)
    outs = []
    for li, n in enumerate((3, 4, 6, 3)):
        for b in range(n):
            pre = 'body.layers.%d.%d' % (li + 1, b)
            s = 2 if (b == 0 and li > 0) else 1
            y = _cu(P, x, pre + '.downsample', s, 0, relu=False) if (pre + '.downsample.conv.weight') in P else x
            t = _cu(P, x, pre + '.u1')
            t = _cu(P, t, pre + '.u2', s, 1)
            x = _cu(P, t, pre + '.u3', add=y)
        outs.append(x)
    return outs


def fpn(P, C):
    """FeaturePyramidNetwork.forward (rcnn.py:23-31) -> P2..P6."""
    n = len(C)
    Ps = [F.conv2d(C[i], P['fpn.conv_laterals.%d.conv.weight' % i], P['fpn.conv_laterals.%d.conv.bias' % i])
          for i in range(n)]
    for i in range(n - 1)[::-1]:
        Ps[i] += F.interpolate(Ps[i + 1], size=Ps[i].shape[2:], mode='nearest')
    for i in range(n):
        Ps[i] = F.conv2d(Ps[i], P['fpn.conv_smooths.%d.conv.weight' % i], P['fpn.conv_smooths.%d.conv.bias' % i],
                         1, 1)
    Ps.append(F.max_pool2d(Ps[-1], 1, stride=2))
    return Ps


def rpn_head(P, x):
    """RegionProposalNetwork.head (rcnn.py:42-47): reg [n, h*w*3, 4], log [n, h*w*3, 1]."""
    n = x.shape[0]
    x = F.relu(F.conv2d(x, P['rpn.conv.conv.weight'], P['rpn.conv.conv.bias'], 1, 1))
    reg = F.conv2d(x, P['rpn.reg.weight'], P['rpn.reg.bias']).permute(0, 2, 3, 1).reshape(n, -1, 4)
    log = F.conv2d(x, P['rpn.log.weight'], P['rpn.log.bias']).permute(0, 2, 3, 1).reshape(n, -1, 1)
    return reg, log


def priors(hw):
    """get_priors(hw, bases, 'corner', 'as_is', concat=False) (anchor.py:20-64)."""
    h, w = hw
    out = []
    for stride, anc in zip(STRIDES, anchors()):
        nx, ny = math.ceil(w / stride), math.ceil(h / stride)
        xs = torch.arange(nx, dtype=torch.float32) * stride
        ys = torch.arange(ny, dtype=torch.float32) * stride
        c = torch.dstack(torch.meshgrid(xs, ys, indexing='xy')).reshape(-1, 2)
        c = c.repeat_interleave(len(anc), dim=0)
        s = torch.tensor(anc, dtype=torch.float32).repeat(nx * ny, 1)
        out.append(torch.hstack([c, s]))
    return out


def decode(pred, pri, mults=(1, 1)):
    """decode_boxes(mode='rcnn', clamp=False) (bbox.py:6-27)."""
    mxy, mwh = mults
    xys = pri[..., 2:] * mxy * pred[..., :2] + pri[..., :2]
    whs = pri[..., 2:] * torch.exp(mwh * pred[..., 2:])
    return torch.cat([xys - whs / 2, xys + whs / 2], dim=-1)


def clamp_to_canvas(boxes, imsizes, imidx):
    """bbox.py:45-49"""
    mx = torch.tensor(imsizes).flip(1).repeat(1, 2)[imidx, :]
    return boxes.clamp_(min=torch.tensor(0), max=mx)


def remove_small(boxes, min_size, *args):
    """bbox.py:52-60"""
    boxes = boxes.view(-1, 4)
    ws = boxes[:, 2] - boxes[:, 0]
    hs = boxes[:, 3] - boxes[:, 1]
    mask = (ws > min_size) & (hs > min_size)
    if torch.count_nonzero(mask) < boxes.shape[0]:
        boxes = boxes[mask]
        args = [t[mask] for t in args]
    return [boxes.reshape(-1, 4), *args]


def rpn(P, fmaps, pri, imsizes):
    """RegionProposalNetwork.forward (rcnn.py:49-82) -> proposals [m,4], imidx [m]."""
    regs, logs = zip(*[rpn_head(P, x) for x in fmaps])
    return rpn_select(regs, logs, pri, imsizes)


def _fma32(a, b, c):
    return (np.asarray(a, np.float64) * np.asarray(b, np.float64) + np.asarray(c, np.float64)).astype(np.float32)


def sleef_expf_u10(d):
    """Sleef_expf16_u10 (AVX512 build inside libtorch_cpu.so, disassembled; Horner with fma,
    2^q applied as two exact power-of-two products)"""
    f = np.float32
    d = np.asarray(d, np.float32)
    q = np.rint((d * f(1.44269502162933349609375)).astype(np.float32)).astype(np.int32)
    qf = q.astype(np.float32)
    s = _fma32(qf, f(-0.693145751953125), d)
    s = _fma32(qf, f(-1.428606765330187045e-06), s)
    u = np.full_like(d, f(0.000198527617612853646278381))
    for c in (0.00139304355252534151077271, 0.00833336077630519866943359, 0.0416664853692054748535156,
              0.166666671633720397949219, 0.5):
        u = _fma32(s, u, f(c))
    u = (_fma32((s * s).astype(np.float32), u, s) + f(1)).astype(np.float32)
    h = q >> 1
    u = (u * np.exp2(h.astype(np.float64)).astype(np.float32)).astype(np.float32)
    u = (u * np.exp2((q - h).astype(np.float64)).astype(np.float32)).astype(np.float32)
    u = np.where(d < -104, f(0), u)
    return np.where(d > 100, f(np.inf), u).astype(np.float32)


def torch_sigmoid_survey(x, threads=8):
    """torch.sigmoid of a contiguous float32 tensor exactly as torch 2.10 computes it on the
    survey container's CPU (AVX512 capability, `threads` intra-op threads): 1 / (1 + exp(-x))
    with Sleef_expf16_u10 on the 32-element vector steps of each parallel_for chunk and glibc
    expf on each chunk's last (len % 32) elements (scripts/torch_sigmoid_order.py checks it
    against torch bit for bit).  Used by rpn_select so that the GPU box's own torch build and
    CPU (vector width, thread count) do not enter the oracle."""
    import ctypes
    x = np.ascontiguousarray(np.asarray(x, np.float32).ravel())
    n = x.size
    f = np.float32
    out = (f(1) / (f(1) + sleef_expf_u10(f(0) - x)).astype(np.float32)).astype(np.float32)
    if n == 0:
        return out
    libm = ctypes.CDLL('libm.so.6')
    libm.expf.restype, libm.expf.argtypes = ctypes.c_float, [ctypes.c_float]
    nt = min(threads, -(-n // 32768))
    cs = -(-n // nt)
    for c0 in range(0, n, cs):
        c1 = min(n, c0 + cs)
        for i in range(c1 - (c1 - c0) % 32, c1):
            out[i] = f(1) / f(f(1) + f(libm.expf(float(-x[i]))))
    return out


def rpn_select(regs, logs, pri, imsizes):
    """filt_dec + sigmoid + clamp + remove_small + batched_nms(0.7) + top-1000 per image
    (rcnn.py:49-82) from the head outputs."""
    n = regs[0].shape[0]
    boxes, logits, lvlen = [], [], []
    for reg, log, p in zip(regs, logs, pri):
        log, top = log.topk(min(1000, log.shape[1]), dim=1)
        reg = reg.gather(1, top.expand(-1, -1, 4))
        pp = p.expand(n, -1, -1).gather(1, top.expand(-1, -1, 4))
        boxes.append(decode(reg, pp))
        logits.append(log)
        lvlen.append(log.shape[1])
    boxes = torch.cat(boxes, axis=1)
    cat = torch.cat(logits, axis=1)
    obj = torch.from_numpy(torch_sigmoid_survey(cat.numpy())).reshape(cat.shape)
    dim = boxes.shape[1]
    boxes, obj = boxes.reshape(-1, 4), obj.flatten()
    idx = torch.nonzero(obj >= 0).squeeze(1)
    boxes, obj = boxes[idx], obj[idx]
    imidx = idx.div(dim, rounding_mode='floor')
    boxes = clamp_to_canvas(boxes, imsizes, imidx)
    boxes, obj, idx, imidx = remove_small(boxes, 0, obj, idx, imidx)
    lv = torch.bucketize(idx % dim, torch.tensor(lvlen).cumsum(0), right=True)
    groups = imidx * 10 + lv
    keep = onms.batched_nms(boxes, obj, groups, 0.7)
    keep = torch.cat([keep[imidx[keep] == i][:1000] for i in range(n)])
    return boxes[keep], imidx[keep]


def roi_align(fmap, rois, out=7, scale=1.0, aligned=True):
    """torchvision.ops.roi_align(fmap [N,C,H,W], rois [R,5] (img, x1, y1, x2, y2), out,
    scale, sampling_ratio=0, aligned) restated per RoI from the published CPU kernel, fp32
    with the C++ evaluation order (no fused multiply-adds)."""
    N, C, H, W = fmap.shape
    R = rois.shape[0]
    res = torch.zeros((R, C, out, out), dtype=torch.float32)
    f32 = np.float32
    off = f32(0.5) if aligned else f32(0.0)
    sc = f32(scale)
    rn = rois.numpy().astype(np.float32)
    fm = fmap.numpy()
    bins = np.arange(out, dtype=np.float32)
    for r in range(R):
        b = int(rn[r, 0])
        x0 = f32(rn[r, 1] * sc - off)
        y0 = f32(rn[r, 2] * sc - off)
        x1 = f32(rn[r, 3] * sc - off)
        y1 = f32(rn[r, 4] * sc - off)
        rw, rh = f32(x1 - x0), f32(y1 - y0)
        if not aligned:
            rw, rh = max(rw, f32(1)), max(rh, f32(1))
        bh, bw = f32(rh / f32(out)), f32(rw / f32(out))
        gh, gw = int(math.ceil(f32(rh / f32(out)))), int(math.ceil(f32(rw / f32(out))))
        cnt = f32(max(gh * gw, 1))
        img = fm[b]
        acc = np.zeros((C, out, out), np.float32)
        # one sample (iy, ix) of every bin (ph, pw) at a time: per-bin accumulation order
        # is the kernel's (iy outer, ix inner)
        ybase = (y0 + bins * bh).astype(np.float32)
        xbase = (x0 + bins * bw).astype(np.float32)
        for iy in range(gh):
            yv = (ybase + f32(f32(f32(iy + 0.5) * bh) / f32(gh))).astype(np.float32)
            for ix in range(gw):
                xv = (xbase + f32(f32(f32(ix + 0.5) * bw) / f32(gw))).astype(np.float32)
                y = np.repeat(yv[:, None], out, 1)
                x = np.repeat(xv[None, :], out, 0)
                empty = (y < -1.0) | (y > H) | (x < -1.0) | (x > W)
                y = np.where(y <= 0, f32(0), y)
                x = np.where(x <= 0, f32(0), x)
                yl = y.astype(np.int64)
                xl = x.astype(np.int64)
                ytop = yl >= H - 1
                xtop = xl >= W - 1
                yl = np.where(ytop, H - 1, yl)
                xl = np.where(xtop, W - 1, xl)
                yh = np.where(ytop, H - 1, yl + 1)
                xh = np.where(xtop, W - 1, xl + 1)
                y = np.where(ytop, yl.astype(np.float32), y)
                x = np.where(xtop, xl.astype(np.float32), x)
                ly = (y - yl.astype(np.float32)).astype(np.float32)
                lx = (x - xl.astype(np.float32)).astype(np.float32)
                hy = (f32(1) - ly).astype(np.float32)
                hx = (f32(1) - lx).astype(np.float32)
                w1, w2, w3, w4 = hy * hx, hy * lx, ly * hx, ly * lx
                w1, w2, w3, w4 = [np.where(empty, f32(0), w).astype(np.float32) for w in (w1, w2, w3, w4)]
                yl, yh, xl, xh = [np.where(empty, 0, t) for t in (yl, yh, xl, xh)]
                v = ((w1 * img[:, yl, xl] + w2 * img[:, yl, xh]) + w3 * img[:, yh, xl]) + w4 * img[:, yh, xh]
                acc = (acc + v).astype(np.float32)
        res[r] = torch.from_numpy(acc / cnt)
    return res


def assign_levels(boxes):
    """assign_fpn_levels (roi.py:7-16) for strides 4..32."""
    ws = boxes[:, 2] - boxes[:, 0]
    hs = boxes[:, 3] - boxes[:, 1]
    k = 4 + torch.log2(torch.sqrt(ws * hs) / 224)
    k = torch.clamp(k, min=2.0, max=5.0)
    return (k - 2.0).to(torch.int64)


def roi_maps(props, imidx, fmaps):
    """roi_align_multilevel (roi.py:19-32) -> [R, 256, 7, 7]."""
    lv = assign_levels(props)
    imboxes = torch.hstack([imidx.unsqueeze(-1).to(props.dtype), props])
    maps = torch.zeros((len(lv), fmaps[0].shape[1], 7, 7))
    for level in range(4):
        idx = torch.nonzero(lv == level).squeeze(1)
        if idx.numel():
            maps[idx] = roi_align(fmaps[level], imboxes[idx], 7, 1 / STRIDES[level], True)
    return maps


def roi_head(P, props, imidx, fmaps, imsizes, n):
    """RoIProcessingNetwork.forward (rcnn.py:103-124)."""
    x = roi_maps(props, imidx, fmaps).flatten(start_dim=1)
    for i in range(2):
        x = F.relu(F.linear(x, P['roi.fc.%d.weight' % i], P['roi.fc.%d.bias' % i]))
    reg = F.linear(x, P['roi.reg.weight'], P['roi.reg.bias']).reshape(x.shape[0], -1, 4)
    log = F.linear(x, P['roi.cls.weight'], P['roi.cls.bias'])
    scr = F.softmax(log, dim=-1)[:, :-1]
    cls = torch.arange(log.shape[1]).view(1, -1).expand_as(log)[:, :-1]
    dim = reg.shape[1]
    reg, scr, cls = reg.reshape(-1, 4), scr.flatten(), cls.flatten()
    fidx = torch.nonzero(scr > 0.05).squeeze(1)
    reg, scr, cls = reg[fidx], scr[fidx], cls[fidx]
    idx = fidx.div(dim, rounding_mode='floor')
    pr, imi = props[idx].clone(), imidx[idx]
    pr[..., 2:] -= pr[..., :2]
    pr[..., :2] += pr[..., 2:] * 0.5
    boxes = decode(reg, pr, (0.1, 0.2))
    boxes = clamp_to_canvas(boxes, imsizes, imi)
    boxes, scr, cls, imi = remove_small(boxes, 0, scr, cls, imi)
    res = []
    for i in range(n):
        m = imi == i
        bi, si, ci = boxes[m], scr[m], cls[m]
        keep = onms.batched_nms(bi, si, ci, 0.5)[:100]
        res.append((bi[keep], si[keep], ci[keep]))
    return [list(t) for t in zip(*res)]


def params_t(params):
    return {k: torch.from_numpy(np.asarray(v)) for k, v in params.items()}


def net(params, x):
    """body + FPN on a preprocessed batch -> P2..P6."""
    P = params_t(params)
    with torch.inference_mode():
        return fpn(P, body(P, x))


def forward(params, frames):
    """FasterRCNN.forward (rcnn.py:141-151): -> (boxes list, scores list, classes list)."""
    P = params_t(params)
    x, so, su = preprocess(frames)
    with torch.inference_mode():
        pri = priors(x.shape[2:])
        xs = fpn(P, body(P, x))
        p, imidx = rpn(P, xs, pri, su)
        n = int(imidx.max()) + 1
        b, s, c = roi_head(P, p, imidx, xs[:-1], su, n)
        scales = (torch.tensor(so) / torch.tensor(su)).flip(1).repeat(1, 2)
        b = [b[i] * scales[i] for i in range(len(b))]
    return [t.numpy() for t in b], [t.numpy() for t in s], [t.numpy() for t in c]

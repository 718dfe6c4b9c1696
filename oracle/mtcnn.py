"""ORACLE — TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline leg).

CPU restatement of the reference MTCNN detector forward
(src/videotofaces/detectors/mtcnn.py) with torch-CPU functional ops, so that it runs on
the GPU box without any reference code.  Every step cites the reference line it follows.
NMS goes through oracle/nms.py (torchvision restatement).  Parity of this restatement with
the reference modules themselves is pinned by tests/golden/*.npz (made by
tests/golden/make_golden.py in the survey container, where the reference imports).
"""
import numpy as np
import torch
import torch.nn.functional as F

from . import nms as onms


def _t(p, name):
    return torch.from_numpy(np.asarray(p[name], np.float32))


def pnet(p, x):
    """mtcnn.py:27-38 -> (reg [B,4,ph,pw], prob [B,ph,pw])"""
    x = F.prelu(F.conv2d(x, _t(p, 'pnet.conv1.weight'), _t(p, 'pnet.conv1.bias')), _t(p, 'pnet.prelu1.weight'))
    x = F.max_pool2d(x, 2, 2, ceil_mode=True)
    x = F.prelu(F.conv2d(x, _t(p, 'pnet.conv2.weight'), _t(p, 'pnet.conv2.bias')), _t(p, 'pnet.prelu2.weight'))
    x = F.prelu(F.conv2d(x, _t(p, 'pnet.conv3.weight'), _t(p, 'pnet.conv3.bias')), _t(p, 'pnet.prelu3.weight'))
    a = F.softmax(F.conv2d(x, _t(p, 'pnet.conv4_1.weight'), _t(p, 'pnet.conv4_1.bias')), dim=1)
    b = F.conv2d(x, _t(p, 'pnet.conv4_2.weight'), _t(p, 'pnet.conv4_2.bias'))
    return b, a[:, 1]


def rnet(p, x):
    """mtcnn.py:58-76"""
    x = F.prelu(F.conv2d(x, _t(p, 'rnet.conv1.weight'), _t(p, 'rnet.conv1.bias')), _t(p, 'rnet.prelu1.weight'))
    x = F.max_pool2d(x, 3, 2, ceil_mode=True)
    x = F.prelu(F.conv2d(x, _t(p, 'rnet.conv2.weight'), _t(p, 'rnet.conv2.bias')), _t(p, 'rnet.prelu2.weight'))
    x = F.max_pool2d(x, 3, 2, ceil_mode=True)
    x = F.prelu(F.conv2d(x, _t(p, 'rnet.conv3.weight'), _t(p, 'rnet.conv3.bias')), _t(p, 'rnet.prelu3.weight'))
    x = x.permute(0, 3, 2, 1).contiguous()
    x = x.reshape(x.shape[0], int(np.prod(x.shape[1:])))
    x = F.prelu(F.linear(x, _t(p, 'rnet.dense4.weight'), _t(p, 'rnet.dense4.bias')), _t(p, 'rnet.prelu4.weight'))
    a = F.softmax(F.linear(x, _t(p, 'rnet.dense5_1.weight'), _t(p, 'rnet.dense5_1.bias')), dim=1)
    b = F.linear(x, _t(p, 'rnet.dense5_2.weight'), _t(p, 'rnet.dense5_2.bias'))
    return b, a[:, 1]


def onet(p, x):
    """mtcnn.py:101-121"""
    x = F.prelu(F.conv2d(x, _t(p, 'onet.conv1.weight'), _t(p, 'onet.conv1.bias')), _t(p, 'onet.prelu1.weight'))
    x = F.max_pool2d(x, 3, 2, ceil_mode=True)
    x = F.prelu(F.conv2d(x, _t(p, 'onet.conv2.weight'), _t(p, 'onet.conv2.bias')), _t(p, 'onet.prelu2.weight'))
    x = F.max_pool2d(x, 3, 2, ceil_mode=True)
    x = F.prelu(F.conv2d(x, _t(p, 'onet.conv3.weight'), _t(p, 'onet.conv3.bias')), _t(p, 'onet.prelu3.weight'))
    x = F.max_pool2d(x, 2, 2, ceil_mode=True)
    x = F.prelu(F.conv2d(x, _t(p, 'onet.conv4.weight'), _t(p, 'onet.conv4.bias')), _t(p, 'onet.prelu4.weight'))
    x = x.permute(0, 3, 2, 1).contiguous()
    x = x.reshape(x.shape[0], int(np.prod(x.shape[1:])))
    x = F.prelu(F.linear(x, _t(p, 'onet.dense5.weight'), _t(p, 'onet.dense5.bias')), _t(p, 'onet.prelu5.weight'))
    a = F.softmax(F.linear(x, _t(p, 'onet.dense6_1.weight'), _t(p, 'onet.dense6_1.bias')), dim=1)
    b = F.linear(x, _t(p, 'onet.dense6_2.weight'), _t(p, 'onet.dense6_2.bias'))
    c = F.linear(x, _t(p, 'onet.dense6_3.weight'), _t(p, 'onet.dense6_3.bias'))
    return b, c, a[:, 1]


def preprocess(frames):
    """mtcnn.py:133-139: stack, NCHW, BGR->RGB, (x-127.5)/128 in fp32."""
    x = np.stack(frames)
    x = x.transpose(0, 3, 1, 2)
    x = x[:, [2, 1, 0], :, :]
    x = (x.astype(np.float32) - 127.5) / 128
    return torch.from_numpy(np.ascontiguousarray(x))


def scale_pyramid(H, W, minsize, factor=0.709):
    """mtcnn.py:141-148 (Python doubles, int() truncation)."""
    scales = []
    s = 12.0 / minsize
    while min(H, W) * s >= 12:
        scales.append(s)
        s *= factor
    sizes = [(int(H * s + 1), int(W * s + 1)) for s in scales]
    return scales, sizes


def cropped_candidates(x, imgidx, boxes, size):
    """mtcnn.py:153-163 (per-box Python loop, degenerate boxes skipped)."""
    H, W = x.shape[2:4]
    lst = [torch.zeros([0, x.shape[1], *size])]
    for k in range(boxes.shape[0]):
        x1, y1, x2, y2 = boxes[k]
        x1, y1, x2, y2 = max(1, int(x1)), max(1, int(y1)), min(W, int(x2)), min(H, int(y2))
        if y2 > y1 - 1 and x2 > x1 - 1:
            crop = x[imgidx[k], :, y1 - 1: y2, x1 - 1: x2]
            lst.append(F.adaptive_avg_pool2d(crop, size).unsqueeze(0))
    return torch.cat(lst)


def refine_bbox(boxes, pred, plus_one=False):
    """mtcnn.py:254-262"""
    w = boxes[:, 2] - boxes[:, 0] + (1 if plus_one else 0)
    h = boxes[:, 3] - boxes[:, 1] + (1 if plus_one else 0)
    b1 = boxes[:, 0] + pred[:, 0] * w
    b2 = boxes[:, 1] + pred[:, 1] * h
    b3 = boxes[:, 2] + pred[:, 2] * w
    b4 = boxes[:, 3] + pred[:, 3] * h
    boxes[:, :4] = torch.stack([b1, b2, b3, b4]).permute(1, 0)
    return boxes


def square_bbox(boxes):
    """mtcnn.py:264-271"""
    h = boxes[:, 3] - boxes[:, 1]
    w = boxes[:, 2] - boxes[:, 0]
    m = torch.max(w, h)
    boxes[:, 0] = boxes[:, 0] + w * 0.5 - m * 0.5
    boxes[:, 1] = boxes[:, 1] + h * 0.5 - m * 0.5
    boxes[:, 2:4] = boxes[:, :2] + m.repeat(2, 1).permute(1, 0)
    return boxes


def nms_iom_chain(boxes, scores, classes, thresh):
    """mtcnn.py:273-309 with method='Min', chain_suppression=True."""
    if boxes.numel() == 0:
        return torch.zeros(0, dtype=torch.int64)
    k = torch.argsort(scores, descending=True)
    classes_sorted = classes[k]
    c = torch.zeros((0, 2), dtype=torch.int64)
    for i in classes.unique():
        ci = torch.combinations(k[classes_sorted == i])
        c = torch.cat((c, ci.reshape(-1, 2)))
    b1 = boxes[c[:, 0]]
    b2 = boxes[c[:, 1]]
    inter_x1 = torch.maximum(b1[:, 0], b2[:, 0])
    inter_y1 = torch.maximum(b1[:, 1], b2[:, 1])
    inter_x2 = torch.minimum(b1[:, 2], b2[:, 2])
    inter_y2 = torch.minimum(b1[:, 3], b2[:, 3])
    inter_w = inter_x2 - inter_x1 + 1
    inter_h = inter_y2 - inter_y1 + 1
    idx = (inter_w > 0) * (inter_h > 0)
    c, b1, b2, inter_w, inter_h = c[idx], b1[idx], b2[idx], inter_w[idx], inter_h[idx]
    inter = inter_w * inter_h
    area1 = (b1[:, 2] - b1[:, 0] + 1) * (b1[:, 3] - b1[:, 1] + 1)
    area2 = (b2[:, 2] - b2[:, 0] + 1) * (b2[:, 3] - b2[:, 1] + 1)
    iom = inter / torch.minimum(area1, area2)
    c = c[iom > thresh]
    dropped = set(c[:, 1].tolist())
    return torch.tensor([i for i in k.tolist() if i not in dropped], dtype=torch.int64)


def stage1(p, x, minsize, trace=None):
    """mtcnn.py:169-208: pyramid, PNet, per-level NMS, cross-level NMS, refine, square."""
    H, W = x.shape[2:4]
    scales, sizes = scale_pyramid(H, W, minsize)
    boxes, scores, imgidx, preds = [], [], [], []
    for i in range(len(scales)):
        xi = F.adaptive_avg_pool2d(x, sizes[i])
        pred, prob = pnet(p, xi)
        mask = prob >= 0.6
        mask_inds = mask.nonzero()
        scores_i = prob[mask]
        imgidx_i = mask_inds[:, 0]
        preds_i = pred.permute(1, 0, 2, 3)[:, mask].permute(1, 0)
        bb = mask_inds[:, 1:].flip(1)
        q1 = ((2 * bb + 1) / scales[i]).floor()
        q2 = ((2 * bb + 12 - 1 + 1) / scales[i]).floor()
        boxes_i = torch.cat([q1, q2], dim=1)
        pick = onms.batched_nms(boxes_i, scores_i, imgidx_i, 0.5)
        if trace is not None:
            trace.append(dict(level=i, nz=int(scores_i.numel()), kept=int(pick.numel())))
        boxes.append(boxes_i[pick])
        preds.append(preds_i[pick])
        scores.append(scores_i[pick])
        imgidx.append(imgidx_i[pick])
    boxes, scores = torch.cat(boxes), torch.cat(scores)
    preds, imgidx = torch.cat(preds), torch.cat(imgidx)
    pick = onms.batched_nms(boxes, scores, imgidx, 0.7)
    boxes, preds, imgidx, scores = boxes[pick], preds[pick], imgidx[pick], scores[pick]
    boxes = refine_bbox(boxes, preds, False)
    boxes = square_bbox(boxes)
    return boxes, imgidx, scores


def forward(p, frames, minsize=20, return_landmarks=False, trace=None):
    """MTCNN.forward mtcnn.py:167-252 -> list of [n_i, 5] float32 per image."""
    with torch.inference_mode():
        x = preprocess(frames)
        boxes, imgidx, _ = stage1(p, x, minsize, trace)
        # stage 2 mtcnn.py:213-222
        proposals = cropped_candidates(x, imgidx, boxes, (24, 24))
        preds, scores = rnet(p, proposals)
        ipass = scores > 0.7
        boxes, scores, preds, imgidx = boxes[ipass, :], scores[ipass], preds[ipass, :], imgidx[ipass]
        pick = onms.batched_nms(boxes, scores, imgidx, 0.7)
        boxes, preds, imgidx = boxes[pick], preds[pick], imgidx[pick]
        boxes = refine_bbox(boxes, preds, True)
        boxes = square_bbox(boxes)
        if trace is not None:
            trace.append(dict(stage=2, n=int(proposals.shape[0]), kept=int(pick.numel())))
        # stage 3 mtcnn.py:228-242
        refinements = cropped_candidates(x, imgidx, boxes, (48, 48))
        preds, landmarks, scores = onet(p, refinements)
        ipass = scores > 0.7
        boxes, scores, preds, imgidx = boxes[ipass, :], scores[ipass], preds[ipass, :], imgidx[ipass]
        landmarks = landmarks[ipass, :]
        w_i = boxes[:, 2] - boxes[:, 0] + 1
        h_i = boxes[:, 3] - boxes[:, 1] + 1
        lm_x = w_i.unsqueeze(1) * landmarks[:, :5] + boxes[:, 0].unsqueeze(1) - 1
        lm_y = h_i.unsqueeze(1) * landmarks[:, 5:] + boxes[:, 1].unsqueeze(1) - 1
        landmarks = torch.stack([lm_x, lm_y], dim=-1)
        boxes = refine_bbox(boxes, preds, True)
        pick = nms_iom_chain(boxes, scores, imgidx, 0.7)
        boxes, scores, landmarks, imgidx = boxes[pick], scores[pick], landmarks[pick], imgidx[pick]
        if trace is not None:
            trace.append(dict(stage=3, n=int(refinements.shape[0]), kept=int(pick.numel())))
        res, ldm = [], []
        for k in range(x.shape[0]):
            idx = imgidx == k
            res.append(torch.cat((boxes[idx], scores[idx].unsqueeze(1)), dim=1).numpy())
            ldm.append(landmarks[idx].numpy())
    if return_landmarks:
        return res, ldm
    return res

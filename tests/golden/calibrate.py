"""Calibrate the synthetic MTCNN face-logit biases; `encoders`, `yolo`, `rcnn`
for the other models' calibrations.

Random weights make the MTCNN gates meaningless, so each face-logit head's bias
difference is chosen so that a fixed fraction of candidates pass its gate on synthetic 720p
frames (min_face_size=5, the RealMTCNN default):
  PNet  prob >= 0.6 : ~0.2% of cells (logit >= ln(0.6/0.4))
  RNet  prob >  0.7 : ~5% of stage-2 proposals
  ONet  prob >  0.7 : ~25% of stage-3 refinements
Run in the survey container; paste the printed values into synth.MTCNN_CALIB.
Uses only the build's own oracle (no reference code).
"""
import math
import sys
import os

import numpy as np
import torch
import torch.nn.functional as F

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'video-to-faces_amd')]
from videotofaces import synth  # noqa: E402
from oracle import mtcnn as om  # noqa: E402


def logit_diff_threshold(d, frac, gate):
    """bias diff b such that fraction `frac` of (d + b) clears the logit gate."""
    q = float(torch.quantile(d.double(), 1.0 - frac))
    return gate - q


def _rnet_hidden(p, x):
    """RNet up to dense4 + PReLU (mtcnn.py:58-70): the 128-d input of the face head"""
    t = om._t
    x = F.prelu(F.conv2d(x, t(p, 'rnet.conv1.weight'), t(p, 'rnet.conv1.bias')), t(p, 'rnet.prelu1.weight'))
    x = F.max_pool2d(x, 3, 2, ceil_mode=True)
    x = F.prelu(F.conv2d(x, t(p, 'rnet.conv2.weight'), t(p, 'rnet.conv2.bias')), t(p, 'rnet.prelu2.weight'))
    x = F.max_pool2d(x, 3, 2, ceil_mode=True)
    x = F.prelu(F.conv2d(x, t(p, 'rnet.conv3.weight'), t(p, 'rnet.conv3.bias')), t(p, 'rnet.prelu3.weight'))
    x = x.permute(0, 3, 2, 1).contiguous().reshape(x.shape[0], -1)
    return F.prelu(F.linear(x, t(p, 'rnet.dense4.weight'), t(p, 'rnet.dense4.bias')), t(p, 'rnet.prelu4.weight'))


def _onet_hidden(p, x):
    """ONet up to dense5 + PReLU (mtcnn.py:101-115): the 256-d input of the face head"""
    t = om._t
    x = F.prelu(F.conv2d(x, t(p, 'onet.conv1.weight'), t(p, 'onet.conv1.bias')), t(p, 'onet.prelu1.weight'))
    x = F.max_pool2d(x, 3, 2, ceil_mode=True)
    x = F.prelu(F.conv2d(x, t(p, 'onet.conv2.weight'), t(p, 'onet.conv2.bias')), t(p, 'onet.prelu2.weight'))
    x = F.max_pool2d(x, 3, 2, ceil_mode=True)
    x = F.prelu(F.conv2d(x, t(p, 'onet.conv3.weight'), t(p, 'onet.conv3.bias')), t(p, 'onet.prelu3.weight'))
    x = F.max_pool2d(x, 2, 2, ceil_mode=True)
    x = F.prelu(F.conv2d(x, t(p, 'onet.conv4.weight'), t(p, 'onet.conv4.bias')), t(p, 'onet.prelu4.weight'))
    x = x.permute(0, 3, 2, 1).contiguous().reshape(x.shape[0], -1)
    return F.prelu(F.linear(x, t(p, 'onet.dense5.weight'), t(p, 'onet.dense5.bias')), t(p, 'onet.prelu5.weight'))


def _face_head(h, large, frac, gate):
    """A face head (2 x C logits) whose logit difference is g * (w . h) + b: w = the Fisher
    direction separating the features of large-box crops from small-box ones (pooled
    covariance, ridge 1e-3 * mean eigenvalue), g = 3 / std, b such that a fraction `frac` of
    the crops clears the gate logit.  Returns (weight [2, C], bias [2]) as float32."""
    hd = h.double().numpy()
    m1, m0 = hd[large].mean(0), hd[~large].mean(0)
    S = np.cov(hd[large].T) + np.cov(hd[~large].T)
    S += 1e-3 * np.trace(S) / len(S) * np.eye(len(S))
    w = np.linalg.solve(S, m1 - m0)
    w /= np.linalg.norm(w)
    u = hd @ w
    g = 3.0 / u.std()
    b = gate - float(np.quantile(g * u, 1 - frac))
    W = np.stack([-0.5 * g * w, 0.5 * g * w]).astype(np.float32)
    return W, np.array([-0.5 * b, 0.5 * b], np.float32)


def main(n_frames=2, n_cal=8, large=45.0, frac2=0.06, frac3=0.5):
    """PNet: the face-logit bias lets ~0.2% of level-0 cells pass the 0.6 gate (MTCNN_CALIB).
    RNet / ONet: random heads pass boxes regardless of content, and with min_face_size 5 almost
    every stage-1 box is a 5-10 px level-0 window, so the detector would report 5 px "faces"
    that the reference's det_min_size=50 (main.py:18) rejects.  The heads are set the way a
    trained MTCNN behaves on these frames: they prefer crops of face-sized boxes.  On n_cal
    synthetic 720p frames (seed 7, not a test seed) each head gets the Fisher direction that
    separates the hidden features of crops of boxes >= `large` px from smaller ones, and a bias
    passing a fraction frac2 (RNet, of stage-2 proposals) / frac3 (ONet, of refinements) of the
    crops.  Written to videotofaces/calib_mtcnn_heads.npz (synth.MTCNN_CALIB uses it)."""
    from oracle import nms as onms
    fr = synth.make_frames(n_frames, seed=0)
    synth.MTCNN_CALIB['face_bias'] = {}
    p = synth.make_params('mtcnn', calibrated=False)
    x = om.preprocess(list(fr))
    # PNet head: d = (w1 - w0) . features
    scales, sizes = om.scale_pyramid(720, 1280, 5)
    xi = F.adaptive_avg_pool2d(x, sizes[0])
    p2 = dict(p)
    p2['pnet.conv4_1.weight'] = np.stack([np.zeros_like(p['pnet.conv4_1.weight'][0]),
                                          p['pnet.conv4_1.weight'][1] - p['pnet.conv4_1.weight'][0]])
    p2['pnet.conv4_1.bias'] = np.zeros(2, np.float32)
    _, prob = om.pnet(p2, xi)
    d = torch.logit(prob.flatten().double())
    b_p = logit_diff_threshold(d[::3], 0.002, math.log(0.6 / 0.4))
    print('pnet.conv4_1.bias diff', round(b_p, 4), '(synth.MTCNN_CALIB)')
    synth.MTCNN_CALIB['face_bias'] = {'pnet.conv4_1.bias': round(b_p, 4)}
    p = synth.make_params('mtcnn', calibrated=False)
    for k in ('gain', 'face_bias'):  # regression gains + the PNet bias, without the heads file
        p.update({n: v for n, v in synth.make_params('mtcnn', calibrated=True, heads=False).items()
                  if n in synth.MTCNN_CALIB[k]})
    fc = synth.make_frames(n_cal, seed=7)
    heads = {}
    with torch.inference_mode():
        x = om.preprocess(list(fc))
        boxes, imgidx, _ = om.stage1(p, x, 5)
        prop = om.cropped_candidates(x, imgidx, boxes, (24, 24))
        big = (boxes[:, 2] - boxes[:, 0]).numpy() >= large
        W, bb = _face_head(_rnet_hidden(p, prop), big, frac2, math.log(0.7 / 0.3))
        heads['rnet.dense5_1.weight'], heads['rnet.dense5_1.bias'] = W, bb
        p.update(heads)
        preds, scores = om.rnet(p, prop)
        ip = scores > 0.7
        print('stage 2: %d proposals, %d >= %g px; RNet passes %d (%d of the large ones)'
              % (len(big), int(big.sum()), large, int(ip.sum()), int((ip.numpy() & big).sum())))
        b3, s3, pr3, i3 = boxes[ip], scores[ip], preds[ip], imgidx[ip]
        pick = onms.batched_nms(b3, s3, i3, 0.7)
        b3 = om.square_bbox(om.refine_bbox(b3[pick], pr3[pick], True))
        ref = om.cropped_candidates(x, i3[pick], b3, (48, 48))
        big3 = (b3[:, 2] - b3[:, 0]).numpy() >= large
        W, bb = _face_head(_onet_hidden(p, ref), big3, frac3, math.log(0.7 / 0.3))
        heads['onet.dense6_1.weight'], heads['onet.dense6_1.bias'] = W, bb
    np.savez(synth._MTCNN_HEADS, **heads)
    p = synth.make_params('mtcnn')
    for seed in (7, 1000):
        res = om.forward(p, list(synth.make_frames(4, seed=seed)), minsize=5)
        w = np.concatenate(res)[:, 2] - np.concatenate(res)[:, 0]
        print('seed %d: faces per frame %s, widths p10/p50/p90 %s' % (seed, [len(r) for r in res],
                                                                     np.percentile(w, [10, 50, 90]).round(1)))


def calibrate_yolo(n_frames=2):
    """Row gains and obj bias for the YOLO pred convs.  Darknet's residual stacks grow the
    bridge activations to O(1e3-1e4), so every row is normalised by its measured std:
    regression/cls rows to std 0.3 (cls bias +3 -> sigmoid ~0.95), and the obj row so that
    0.5% of priors reach obj >= 0.005 (logit -5.2933, into NMS) and 0.05% reach obj > 0.5
    (logit 0, survive a 0.4 score filter), pooled over the 3 levels."""
    from oracle import yolo as oy
    fr = synth.make_frames(n_frames, seed=0)
    synth.YOLO_CALIB['row_gain'] = {r: 1.0 for r in range(6)}
    synth.YOLO_CALIB['row_bias'] = {}
    p = synth.make_params('yolo')
    for i in range(3):
        p['head.convs_pred.%d.bias' % i][:] = 0.0
    x, _, _ = oy.preprocess(list(fr))
    maps = oy.net(p, x)
    gains = {}
    for r in range(6):
        d = torch.cat([m[:, r::6].flatten() for m in maps]).double()
        gains[r] = float('%.6g' % (0.3 / float(d.std())))
        if r == 4:
            q1, q2 = float(torch.quantile(d, 1 - 0.005)), float(torch.quantile(d, 1 - 0.0005))
            g = 5.2933 / (q2 - q1)
            gains[4] = float('%.6g' % g)
            b = float('%.6g' % (-g * q2))
            print('obj raw std %.4f q99.5 %.4f q99.95 %.4f -> gain %.6g bias %.6g' % (float(d.std()), q1, q2, g, b))
    synth.YOLO_CALIB['row_gain'] = gains
    synth.YOLO_CALIB['row_bias'] = {4: b, 5: 3.0}
    p = synth.make_params('yolo')
    bx, sc, _ = oy.forward(p, list(fr))
    print('per frame kept', [len(s) for s in sc], 'score>0.4', [int((s > 0.4).sum()) for s in sc])
    print('box sizes', [np.round(np.median(b[:, 2:] - b[:, :2], 0), 1) for b in bx])
    print('YOLO_CALIB =', synth.YOLO_CALIB)


def calibrate_rcnn(n_frames=2):
    """Gains for the RPN and RoI heads of the Faster R-CNN (rcnn.py:34-124) and the face-class
    bias: RPN logits to std 2, RPN deltas to std 0.1, RoI deltas to std 0.5 (x0.1/x0.2 in
    decode); face score = sigmoid(g*u + c) with ~8% of proposals over 0.05 and ~1% over 0.4."""
    from oracle import rcnn as orc
    fr = synth.make_frames(n_frames, seed=0)
    synth.RCNN_CALIB['gain'] = {}
    synth.RCNN_CALIB['face_bias'] = {}
    p = synth.make_params('rcnn')
    x, so, su = orc.preprocess(list(fr))
    P = orc.params_t(p)
    with torch.inference_mode():
        xs = orc.fpn(P, orc.body(P, x))
        regs, logs = zip(*[orc.rpn_head(P, t) for t in xs])
    lg = torch.cat([t.flatten() for t in logs]).double()
    rg = torch.cat([t.flatten() for t in regs]).double()
    print('feature std per level', [round(float(t.std()), 3) for t in xs])
    g_log = float('%.6g' % (2.0 / float(lg.std())))
    g_reg = float('%.6g' % (0.1 / float(rg.std())))
    synth.RCNN_CALIB['gain'] = {'rpn.log.weight': g_log, 'rpn.reg.weight': g_reg}
    p = synth.make_params('rcnn')
    P = orc.params_t(p)
    with torch.inference_mode():
        props, imidx = orc.rpn(P, xs, orc.priors(x.shape[2:]), su)
        print('proposals', props.shape[0], 'median wh', np.median((props[:, 2:] - props[:, :2]).numpy(), 0))
        f = orc.roi_maps(props, imidx, xs[:-1]).flatten(start_dim=1)
        for i in range(2):
            f = F.relu(F.linear(f, P['roi.fc.%d.weight' % i], P['roi.fc.%d.bias' % i]))
        w = P['roi.cls.weight']
        u = (f @ (w[0] - w[1])).double()
        reg = F.linear(f, P['roi.reg.weight']).double()
    q92, q99 = float(torch.quantile(u, 0.92)), float(torch.quantile(u, 0.99))
    g = (math.log(0.4 / 0.6) - math.log(0.05 / 0.95)) / (q99 - q92)
    c = math.log(0.05 / 0.95) - g * q92
    synth.RCNN_CALIB['gain'].update({'roi.cls.weight': float('%.6g' % g),
                                     'roi.reg.weight': float('%.6g' % (0.5 / float(reg.std())))})
    synth.RCNN_CALIB['face_bias'] = {'roi.cls.bias': float('%.6g' % -c)}
    p = synth.make_params('rcnn')
    bx, sc, _ = orc.forward(p, list(fr))
    print('per frame kept', [len(s) for s in sc], 'score>0.4', [int((s > 0.4).sum()) for s in sc])
    print('RCNN_CALIB =', synth.RCNN_CALIB)


def _blobs(crops, size, scale):
    """cv2.dnn.blobFromImages(crops, scale, (size, size), 127.5, swapRB=True) restated
    (oracle.facenet.resize_linear_u8: the INTER_LINEAR restatement)"""
    from oracle.facenet import resize_linear_u8
    out = []
    for c in crops:
        r = resize_linear_u8(c, size)[:, :, ::-1].transpose(2, 0, 1)
        out.append((torch.from_numpy(np.ascontiguousarray(r)).float() - 127.5) * np.float32(scale))
    return torch.stack(out)


def _spread(X):
    Xn = X / np.linalg.norm(X, axis=1, keepdims=True)
    D = 1 - Xn @ Xn.T
    n = len(X)
    Dm = D + (1 - np.tri(n, k=-1)) * 1e4
    return np.percentile(D[np.tril_indices(n, -1)], [5, 50, 95]), int((~(Dm.min(1) <= 0.25)).sum())


def calibrate_encoders(n_frames=48):
    """FaceNet's final BatchNorm1d running statistics (synth._encoder_calib): the mean and
    variance of its input (Linear 1792->512 output) over the face crops of n_frames synthetic
    720p frames (seed 7 -- not a test seed), written to videotofaces/calib_facenet_bn.npz.
    Also prints the embeddings' cosine-distance spread with and without the calibration, for
    FaceNet and for ViT-L (synth.VIT_QK_GAIN)."""
    import oracle.facenet as ofn
    from oracle.vit import vit
    fr, faces = synth.make_frames(n_frames, seed=7, return_faces=True)
    crops = synth.face_crops(fr, faces)
    x = _blobs(crops, 160, 1 / 128)
    p = synth.make_params('facenet', calibrated=False)
    q = dict(p)
    q['main.9.running_mean'] = np.zeros(512, np.float32)
    q['main.9.running_var'] = np.full(512, 1 - 1e-3, np.float32)
    q['main.9.weight'] = np.ones(512, np.float32)
    q['main.9.bias'] = np.zeros(512, np.float32)
    norm = ofn.F.normalize
    ofn.F.normalize = lambda t, p=2, dim=1: t
    try:
        feat = ofn.inception_resnet_v1(q, x).numpy().astype(np.float64)
    finally:
        ofn.F.normalize = norm
    mean, var = feat.mean(0).astype(np.float32), feat.var(0).astype(np.float32)
    np.savez(synth._FACENET_BN, mean=mean, var=var, n_crops=np.array(len(crops)), seed=np.array(7))
    print('facenet BN1d input: %d crops, |mean| %.3f, mean std %.4f' % (len(crops), np.linalg.norm(mean),
                                                                      np.sqrt(var).mean()))
    for tag, prm in (('uncalibrated', p), ('calibrated', synth.make_params('facenet'))):
        pct, keep = _spread(ofn.inception_resnet_v1(prm, x).numpy())
        print('facenet %s: cosine distance p5/p50/p95 %s, dedupe(0.25) keeps %d / %d'
              % (tag, np.round(pct, 4), keep, len(crops)))
    xv = _blobs(crops[:64], 128, 1 / 127.5)
    for tag, prm in (('uncalibrated', synth.make_params('vit_l', calibrated=False)),
                     ('q/k gain %g' % synth.VIT_QK_GAIN, synth.make_params('vit_l'))):
        pct, keep = _spread(vit(prm, xv, 1024, 24).numpy())
        print('vit_l %s: cosine distance p5/p50/p95 %s, dedupe(0.25) keeps %d / %d'
              % (tag, np.round(pct, 4), keep, len(xv)))


if __name__ == '__main__':
    if sys.argv[1:] == ['encoders']:
        calibrate_encoders()
    elif sys.argv[1:] == ['rcnn']:
        calibrate_rcnn()
    elif sys.argv[1:] == ['yolo']:
        calibrate_yolo()
    else:
        main()

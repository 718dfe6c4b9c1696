"""Generate golden vectors from the REFERENCE's own modules (survey container only).

The reference package cannot be imported as-is here (``cv2``/``torchvision`` are absent,
SURVEY.md §8c).  It is loaded under the alias ``ref_vtf`` with import-time shims:
  * ``cv2``: a stub whose attributes raise (model forwards never touch cv2);
  * ``torchvision.ops.batched_nms``: a pure-torch restatement of torchvision's published
    algorithm written here (independent of oracle/nms_oracle.c, so the two cross-check).
Weights are the build's deterministic synthetic weights (videotofaces.synth) loaded with
``load_state_dict(strict=True)``.  Outputs are saved as small .npz fixtures; the reference
never travels to the GPU box, only these arrays do.

    python tests/golden/make_golden.py            # all fixtures
"""
import importlib
import os
import sys
import tempfile
import types

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, 'video-to-faces_amd')]
from videotofaces import synth  # noqa: E402

REF_SRC = '/root/reference/src/videotofaces'


def _tv_nms(boxes, scores, thr):
    # torchvision nms_kernel_impl: stable descending sort, greedy, fp32 IoU vs double thr.
    # The inner loop over j is vectorised with fp32 torch ops (same per-element rounding).
    boxes = boxes.float()
    x1, y1, x2, y2 = boxes.unbind(1)
    areas = (x2 - x1) * (y2 - y1)
    order = torch.sort(scores, stable=True, descending=True)[1]
    n = boxes.shape[0]
    sup = torch.zeros(n, dtype=torch.bool)
    keep = []
    zero = torch.tensor(0, dtype=torch.float32)
    for _i in range(n):
        i = int(order[_i])
        if sup[i]:
            continue
        keep.append(i)
        js = order[_i + 1:]
        js = js[~sup[js]]
        if js.numel() == 0:
            continue
        xx1 = torch.maximum(x1[i], x1[js])
        yy1 = torch.maximum(y1[i], y1[js])
        xx2 = torch.minimum(x2[i], x2[js])
        yy2 = torch.minimum(y2[i], y2[js])
        w = torch.maximum(zero, xx2 - xx1)
        h = torch.maximum(zero, yy2 - yy1)
        inter = w * h
        ovr = inter / ((areas[i] + areas[js]) - inter)
        sup[js[ovr.double() > thr]] = True
    return torch.tensor(keep, dtype=torch.int64)


def _tv_batched_nms(boxes, scores, idxs, thr):
    if boxes.numel() > 4000:
        keep_mask = torch.zeros_like(scores, dtype=torch.bool)
        for class_id in torch.unique(idxs):
            curr = torch.where(idxs == class_id)[0]
            keep_mask[curr[_tv_nms(boxes[curr], scores[curr], thr)]] = True
        keep_indices = torch.where(keep_mask)[0]
        return keep_indices[scores[keep_indices].sort(descending=True)[1]]
    if boxes.numel() == 0:
        return torch.empty((0,), dtype=torch.int64)
    max_coordinate = boxes.max()
    offsets = idxs.to(boxes) * (max_coordinate + torch.tensor(1).to(boxes))
    return _tv_nms(boxes + offsets[:, None], scores, thr)


def _tv_roi_align(input, boxes, output_size, spatial_scale=1.0, sampling_ratio=-1, aligned=False):
    # torchvision roi_align CPU kernel (roi_align_kernel.cpp), restated sample by sample with
    # fp32 scalars (independent of oracle/rcnn.py's bin-vectorised restatement; the two
    # cross-check in tests/test_oracle.py).
    import math
    f32 = np.float32
    ph_n, pw_n = output_size
    N, C, H, W = input.shape
    fm = input.numpy()
    bx = boxes.numpy().astype(np.float32)
    out = np.zeros((bx.shape[0], C, ph_n, pw_n), np.float32)
    off = f32(0.5) if aligned else f32(0)
    sc = f32(spatial_scale)
    for r in range(bx.shape[0]):
        img = fm[int(bx[r, 0])]
        sw, sh = f32(bx[r, 1] * sc - off), f32(bx[r, 2] * sc - off)
        ew, eh = f32(bx[r, 3] * sc - off), f32(bx[r, 4] * sc - off)
        rw, rh = f32(ew - sw), f32(eh - sh)
        if not aligned:
            rw, rh = max(rw, f32(1)), max(rh, f32(1))
        bsh, bsw = f32(rh / f32(ph_n)), f32(rw / f32(pw_n))
        gh = sampling_ratio if sampling_ratio > 0 else int(math.ceil(f32(rh / f32(ph_n))))
        gw = sampling_ratio if sampling_ratio > 0 else int(math.ceil(f32(rw / f32(pw_n))))
        count = f32(max(gh * gw, 1))
        for ph in range(ph_n):
            for pw in range(pw_n):
                val = np.zeros(C, np.float32)
                for iy in range(gh):
                    y = f32(f32(sh + f32(f32(ph) * bsh)) + f32(f32(f32(iy + 0.5) * bsh) / f32(gh)))
                    for ix in range(gw):
                        x = f32(f32(sw + f32(f32(pw) * bsw)) + f32(f32(f32(ix + 0.5) * bsw) / f32(gw)))
                        if y < -1.0 or y > H or x < -1.0 or x > W:
                            w1 = w2 = w3 = w4 = f32(0)
                            p1 = p2 = p3 = p4 = (0, 0)
                        else:
                            yy, xx = (f32(0) if y <= 0 else y), (f32(0) if x <= 0 else x)
                            yl, xl = int(yy), int(xx)
                            if yl >= H - 1:
                                yh = yl = H - 1
                                yy = f32(yl)
                            else:
                                yh = yl + 1
                            if xl >= W - 1:
                                xh = xl = W - 1
                                xx = f32(xl)
                            else:
                                xh = xl + 1
                            ly, lx = f32(yy - f32(yl)), f32(xx - f32(xl))
                            hy, hx = f32(1.0 - float(ly)), f32(1.0 - float(lx))
                            w1, w2, w3, w4 = f32(hy * hx), f32(hy * lx), f32(ly * hx), f32(ly * lx)
                            p1, p2, p3, p4 = (yl, xl), (yl, xh), (yh, xl), (yh, xh)
                        t = (((w1 * img[:, p1[0], p1[1]]).astype(np.float32) + (w2 * img[:, p2[0], p2[1]]))
                             .astype(np.float32) + (w3 * img[:, p3[0], p3[1]])).astype(np.float32)
                        t = (t + (w4 * img[:, p4[0], p4[1]])).astype(np.float32)
                        val = (val + t).astype(np.float32)
                out[r, :, ph, pw] = val / count
    return torch.from_numpy(out)


def load_ref():
    if 'ref_vtf' in sys.modules:
        return sys.modules['ref_vtf']
    cv2 = types.ModuleType('cv2')

    def _absent(name):
        def f(*a, **k):
            raise RuntimeError('cv2.%s is not available in this container' % name)
        return f
    cv2.__getattr__ = _absent
    sys.modules['cv2'] = cv2
    tv = types.ModuleType('torchvision')
    ops = types.ModuleType('torchvision.ops')
    ops.batched_nms = _tv_batched_nms
    ops.nms = _tv_nms
    ops.roi_align = _tv_roi_align
    tv.ops = ops
    sys.modules['torchvision'] = tv
    sys.modules['torchvision.ops'] = ops
    pkg = types.ModuleType('ref_vtf')
    pkg.__path__ = [REF_SRC]
    sys.modules['ref_vtf'] = pkg
    return pkg


def _load(module, params):
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in params.items()}
    module.load_state_dict(sd, strict=True)
    module.eval()
    return module


def gen_mtcnn():
    load_ref()
    m = importlib.import_module('ref_vtf.detectors.mtcnn')
    p = synth.make_params('mtcnn')
    net = _load(m.MTCNN('cpu'), p)
    g = torch.Generator().manual_seed(7)
    out = {}
    with torch.inference_mode():
        x = torch.rand(2, 3, 40, 56, generator=g) * 2 - 1
        reg, prob = net.pnet(x)
        out.update(pnet_in=x.numpy(), pnet_reg=reg.numpy(), pnet_prob=prob.numpy())
        x = torch.rand(5, 3, 24, 24, generator=g) * 2 - 1
        reg, prob = net.rnet(x)
        out.update(rnet_in=x.numpy(), rnet_reg=reg.numpy(), rnet_prob=prob.numpy())
        x = torch.rand(5, 3, 48, 48, generator=g) * 2 - 1
        reg, lm, prob = net.onet(x)
        out.update(onet_in=x.numpy(), onet_reg=reg.numpy(), onet_lm=lm.numpy(), onet_prob=prob.numpy())
        # pyramid resample (MTCNN._resample == adaptive_avg_pool2d), up- and down-sampling
        fr = synth.make_frames(1, 90, 160, seed=3)
        xx = net._preprocess(list(fr), 'cpu')
        out['pyr_frame'] = fr
        scales, sizes = net._scale_pyramid(90, 160, 5, 0.709)
        for i, sz in enumerate(sizes[:4]):
            out['pyr_level%d' % i] = net._resample(xx, sz).numpy()
        out['pyr_sizes'] = np.array(sizes[:4], np.int64)
    # end-to-end: two 720p frames at the RealMTCNN default min_face_size=5, and the
    # reference tests' min_face_size=20 (tests/test_mtcnn.py:17)
    frames = synth.make_frames(2, seed=0)
    out['e2e_frames_seed'] = np.array([0])
    for ms in (5, 20):
        with torch.inference_mode():
            res, ldm = net(list(frames), ms, return_landmarks=True)
        out['e2e_ms%d_counts' % ms] = np.array([r.shape[0] for r in res], np.int64)
        out['e2e_ms%d_boxes' % ms] = np.concatenate(res).astype(np.float32) if sum(r.shape[0] for r in res) else np.zeros((0, 5), np.float32)
        out['e2e_ms%d_landmarks' % ms] = np.concatenate(ldm).astype(np.float32) if len(ldm) else np.zeros((0, 5, 2), np.float32)
    # small frames (fast to check on CPU in the not-gpu suite)
    small = synth.make_frames(3, 144, 256, seed=5)
    out['small_frames'] = small
    with torch.inference_mode():
        res = net(list(small), 5)
    out['small_ms5_counts'] = np.array([r.shape[0] for r in res], np.int64)
    out['small_ms5_boxes'] = np.concatenate(res).astype(np.float32)
    np.savez_compressed(os.path.join(HERE, 'mtcnn.npz'), **out)
    print('mtcnn', {k: v.shape for k, v in out.items()})


def gen_facenet():
    load_ref()
    f = importlib.import_module('ref_vtf.encoders.facenet')
    net = _load(f.InceptionResnetV1('cpu'), synth.make_params('facenet'))
    g = torch.Generator().manual_seed(11)
    # the encoder input after cv2.dnn.blobFromImages(1/128, 160x160, 127.5, swapRB):
    # (u8 - 127.5) / 128 of a uint8 image -> exact values
    u8 = torch.randint(0, 256, (4, 3, 160, 160), generator=g).float()
    x = (u8 - 127.5) * (1 / 128)
    with torch.inference_mode():
        y = net(x)
    np.savez_compressed(os.path.join(HERE, 'facenet.npz'), u8=u8.to(torch.uint8).numpy(), emb=y.numpy())
    print('facenet', y.shape, float(y.norm(dim=1).mean()))


def gen_vit():
    load_ref()
    v = importlib.import_module('ref_vtf.encoders.vit')
    g = torch.Generator().manual_seed(13)
    out = {}
    u8 = torch.randint(0, 256, (2, 3, 128, 128), generator=g)
    x = (u8.float() - 127.5) * np.float32(1 / 127.5)  # blobFromImages(1/127.5, 128x128, 127.5)
    out['u8'] = u8.to(torch.uint8).numpy()
    for name, dim, depth in (('vit_b', 768, 12), ('vit_l', 1024, 24)):
        net = _load(v.ViT('cpu', 128, 16, dim, depth), synth.make_params(name))
        with torch.inference_mode():
            out[name] = net(x if name == 'vit_b' else x[:1]).numpy()
        print(name, out[name].shape, float(np.abs(out[name]).mean()))
    np.savez_compressed(os.path.join(HERE, 'vit.npz'), **out)


def gen_grouping():
    load_ref()
    dupes = importlib.import_module('ref_vtf.dupes')
    grouping = importlib.import_module('ref_vtf.grouping')
    rng = np.random.default_rng(0)
    N, D = 600, 64
    centers = rng.normal(0, 1, (8, D)).astype(np.float32)
    lab = rng.integers(0, 8, N)
    X = (centers[lab] + 1.0 * rng.normal(0, 1, (N, D))).astype(np.float32)
    # plant near-duplicates of earlier rows
    for i in range(20):
        j = rng.integers(1, N)
        k = rng.integers(0, j)
        X[j] = X[k] + 0.01 * rng.normal(0, 1, D).astype(np.float32)
    out = dict(X=X)
    with tempfile.TemporaryDirectory() as td:
        os.makedirs(os.path.join(td, 'faces'))
        names = ['f%05d.jpg' % i for i in range(N)]
        for n in names:
            open(os.path.join(td, 'faces', n), 'w').close()
        Xk, goods = dupes.remove_dupes_overall(X.copy(), names, ('enc', 0.25, False, td))
    out['dedupe_keep'] = np.array([int(n[1:6]) for n in goods], np.int64)
    import sklearn.metrics
    Dm = sklearn.metrics.pairwise.cosine_distances(X)
    Dm += (1 - np.tri(N, k=-1).astype(Dm.dtype)) * 10000
    out['dedupe_mins'] = Dm.min(axis=1)
    out['dedupe_inds'] = Dm.argmin(axis=1)
    # cluster_faces internals (grouping.py:97-116): KMeans + three scores per k
    import sklearn.cluster
    ks = list(range(2, 10))
    labels, scores = [], []
    for k in ks:
        lb = sklearn.cluster.KMeans(n_clusters=k, random_state=0, n_init='auto').fit(Xk).labels_
        labels.append(lb)
        scores.append((sklearn.metrics.silhouette_score(Xk, lb), sklearn.metrics.calinski_harabasz_score(Xk, lb),
                       sklearn.metrics.davies_bouldin_score(Xk, lb)))
    out['kmeans_k'] = np.array(ks)
    out['kmeans_labels'] = np.stack(labels).astype(np.int32)
    out['cluster_scores'] = np.array(scores, np.float64)
    # classify (grouping.py:50-66)
    R = X[[3, 50, 100]] + 0.05
    with tempfile.TemporaryDirectory() as td:
        inds, classes = grouping.classify(X, R, ['a', 'b', 'c'], 0.9, False, [], td)
    out['classify_R'] = R
    out['classify_inds'] = np.asarray(inds, np.int64)
    np.savez_compressed(os.path.join(HERE, 'grouping.npz'), **out)
    print('grouping', {k: v.shape for k, v in out.items()})


def gen_yolo():
    """YOLOv3 (yolo.py:131-176) from the letterboxed tensor on: the reference's preprocess
    calls cv2.resize (absent), so the resized uint8 images are made with the build's
    INTER_LINEAR restatement (oracle/yolo.py, parity-unpinned step) and stored as the
    golden INPUT; to_tensors/pad_and_batch, the net, priors, postprocess and scale_boxes
    are the reference's own code."""
    load_ref()
    y = importlib.import_module('ref_vtf.detectors.yolo')
    prep = importlib.import_module('ref_vtf.detectors.operations.prep')
    sys.path.insert(0, ROOT)
    from oracle import yolo as oy
    net = _load(y.YOLOv3('cpu'), synth.make_params('yolo'))
    frames = synth.make_frames(2, seed=0)
    resized, szo, szu = [], [], []
    for f in frames:
        sz = f.shape[:2]
        scl = min(608 / min(sz), 608 / max(sz))
        n = int(sz[0] * scl + 0.5), int(sz[1] * scl + 0.5)
        resized.append(oy.resize_linear_u8_hw(f, n))
        szo.append(sz)
        szu.append(n)
    with torch.inference_mode():
        ts = prep.to_tensors(resized, 'cpu', None, 255, True)
        x = prep.pad_and_batch(ts, 32)
        xs = net.head(net.neck(net.backbone(x)))
        pri = y.get_priors(x.shape[-2:], y.YOLOv3.bases, 'cpu', 'center')
        b, s, c = net.postprocess(xs, pri, num_classes=1)
        b = y.scale_boxes(b, szo, szu)
    out = dict(resized=np.stack(resized), szo=np.array(szo), szu=np.array(szu),
               counts=np.array([len(t) for t in s], np.int64),
               boxes=torch.cat(b).numpy(), scores=torch.cat(s).numpy(), classes=torch.cat(c).numpy())
    for i, m in enumerate(xs):
        out['map%d' % i] = m.numpy()
    np.savez_compressed(os.path.join(HERE, 'yolo.npz'), **out)
    print('yolo', {k: v.shape for k, v in out.items()}, 'counts', out['counts'])


def gen_kmeans():
    """cluster_faces internals at N=2000, D=512, k=2..16 (grouping.py:97-107) with the
    reference's sklearn (1.7.2 here): KMeans labels and the three scores per k."""
    import hashlib
    import sklearn.cluster
    import sklearn.metrics
    X = synth.planted_clusters()
    ks = list(range(2, 17))
    labels, scores = [], []
    for k in ks:
        lb = sklearn.cluster.KMeans(n_clusters=k, random_state=0, n_init='auto').fit(X).labels_
        labels.append(lb)
        scores.append((sklearn.metrics.silhouette_score(X, lb), sklearn.metrics.calinski_harabasz_score(X, lb),
                       sklearn.metrics.davies_bouldin_score(X, lb)))
    sil = sklearn.metrics.silhouette_samples(X, labels[6])
    np.savez_compressed(os.path.join(HERE, 'kmeans.npz'), X_sha256=np.frombuffer(
        hashlib.sha256(X.tobytes()).digest(), np.uint8), k=np.array(ks), labels=np.stack(labels).astype(np.int8),
        scores=np.array(scores, np.float64), sil_k8=sil.astype(np.float32))
    print('kmeans', X.shape, 'best k', ks[int(np.argmax([s[0] for s in scores]))])


def gen_rcnn():
    """Faster R-CNN (rcnn.py:127-151) from the letterboxed tensor on, with the reference's
    own modules; cv2.resize is the build's INTER_LINEAR restatement (parity-unpinned step,
    pinned here by a hash of the resized images) and roi_align the shim above.
    Also: RPN head maps of a small input (conv-stack parity at tight tolerance) and
    roi_align on random maps with edge-case boxes."""
    import hashlib
    load_ref()
    r = importlib.import_module('ref_vtf.detectors.rcnn')
    prep = importlib.import_module('ref_vtf.detectors.operations.prep')
    bbox = importlib.import_module('ref_vtf.detectors.operations.bbox')
    sys.path.insert(0, ROOT)
    from oracle import yolo as oy
    net = _load(r.FasterRCNN('cpu'), synth.make_params('rcnn'))
    out = {}
    g = torch.Generator().manual_seed(17)
    with torch.inference_mode():
        xs = torch.randn(1, 3, 64, 96, generator=g)
        fm = net.fpn(net.body(xs))
        for i, f in enumerate(fm):
            reg, log = net.rpn.head(f)
            out['small_reg%d' % i] = reg.numpy()
            out['small_log%d' % i] = log.numpy()
        out['small_x'] = xs.numpy()
        # roi_align on random maps (aligned, adaptive grid); boxes cover interior, edges,
        # outside the map, degenerate and large
        fmap = torch.randn(2, 16, 20, 24, generator=g)
        rois = torch.tensor([[0, 3.2, 4.7, 40.1, 33.3], [1, 0, 0, 96, 80], [0, -10, -8, 5, 6],
                             [1, 90, 70, 130, 100], [0, 10, 10, 10.5, 30], [1, 20, 15, 20, 15],
                             [0, 1.3, 2.9, 79.8, 77.7], [1, 50.5, 20.25, 60.75, 41]], dtype=torch.float32)
        out['ra_fmap'], out['ra_rois'] = fmap.numpy(), rois.numpy()
        out['ra_out'] = _tv_roi_align(fmap, rois, (7, 7), 0.25, 0, True).numpy()
    frames = synth.make_frames(2, seed=0)
    resized, szo, szu = [], [], []
    for f in frames:
        sz = f.shape[:2]
        scl = min(800 / min(sz), 1333 / max(sz))
        n = int(sz[0] * scl + 0.5), int(sz[1] * scl + 0.5)
        resized.append(oy.resize_linear_u8_hw(f, n))
        szo.append(sz)
        szu.append(n)
    with torch.inference_mode():
        ts = prep.to_tensors(resized, 'cpu', 'imagenet', 'imagenet', True)
        x = prep.pad_and_batch(ts, 32)
        pri = r.get_priors(x.shape[2:], net.bases, 'cpu', 'corner', 'as_is', concat=False)
        fm = net.fpn(net.body(x))
        p, imidx = net.rpn(fm, pri, szu)
        out['proposals'], out['prop_imidx'] = p.numpy().copy(), imidx.numpy().copy()
        b, s, c = net.roi(p, imidx, fm[:-1], net.strides[:-1], szu)
        b = bbox.scale_boxes(b, szo, szu)
    out.update(resized_sha256=np.frombuffer(hashlib.sha256(np.stack(resized).tobytes()).digest(), np.uint8),
               szo=np.array(szo), szu=np.array(szu), counts=np.array([len(t) for t in s], np.int64),
               boxes=torch.cat(b).numpy(), scores=torch.cat(s).numpy(), classes=torch.cat(c).numpy())
    np.savez_compressed(os.path.join(HERE, 'rcnn.npz'), **out)
    print('rcnn', {k: v.shape for k, v in out.items()}, 'counts', out['counts'])


def gen_dupes():
    """remove_dupes_overall('hash') (dupes.py:51-93) of the reference on 64-bit average-hash
    bit arrays with planted near-duplicates (the cv2 ahash itself is not runnable here)."""
    import sklearn.metrics
    load_ref()
    dupes = importlib.import_module('ref_vtf.dupes')
    rng = np.random.default_rng(21)
    N = 400
    X = rng.integers(0, 2, (N, 64))
    for i in range(60):
        j = int(rng.integers(1, N))
        k = int(rng.integers(0, j))
        X[j] = X[k]
        flip = rng.choice(64, int(rng.integers(0, 12)), replace=False)
        X[j, flip] ^= 1
    with tempfile.TemporaryDirectory() as td:
        os.makedirs(os.path.join(td, 'faces'))
        names = ['f%05d.jpg' % i for i in range(N)]
        for n in names:
            open(os.path.join(td, 'faces', n), 'w').close()
        _, goods = dupes.remove_dupes_overall(X.copy(), names, ('hash', 8, False, td))
    D = sklearn.metrics.pairwise_distances(X, metric=lambda a, b: np.count_nonzero(a != b)).astype(np.uint16)
    D += (1 - np.tri(N, k=-1).astype(D.dtype)) * 10000
    np.savez_compressed(os.path.join(HERE, 'dupes.npz'), X=X.astype(np.uint8), keep=np.array(
        [int(n[1:6]) for n in goods], np.int64), mins=D.min(axis=1), inds=D.argmin(axis=1))
    print('dupes', N, 'kept', len(goods))


def _u8(seed, shape):
    """seeded uint8 test images (numpy PCG64: identical on the GPU box)"""
    return np.random.default_rng(seed).integers(0, 256, shape, dtype=np.uint8)


def _yolo_input(frames):
    """the reference's letterbox input from the build's INTER_LINEAR restatement (cv2 absent)"""
    sys.path.insert(0, ROOT)
    from oracle import yolo as oy
    prep = importlib.import_module('ref_vtf.detectors.operations.prep')
    resized, szo, szu = [], [], []
    for f in frames:
        sz = f.shape[:2]
        scl = min(608 / min(sz), 608 / max(sz))
        n = int(sz[0] * scl + 0.5), int(sz[1] * scl + 0.5)
        resized.append(oy.resize_linear_u8_hw(f, n))
        szo.append(sz)
        szu.append(n)
    ts = prep.to_tensors(resized, 'cpu', None, 255, True)
    return prep.pad_and_batch(ts, 32), szo, szu, resized


def _yolo_ref(net, y, frames):
    with torch.inference_mode():
        x, szo, szu, resized = _yolo_input(frames)
        xs = net.head(net.neck(net.backbone(x)))
        pri = y.get_priors(x.shape[-2:], y.YOLOv3.bases, 'cpu', 'center')
        b, s, _ = net.postprocess(xs, pri, num_classes=1)
        b = y.scale_boxes(b, szo, szu)
    return [t.numpy() for t in b], [t.numpy() for t in s], resized


def gen_shapes():
    """Golden vectors at the benchmarked shapes (BASELINE configs 2-5), from the reference's own
    modules: MTCNN 720p det-batch 16 at min_face_size 5 and det-batch 4 at 20 (main.py:18
    default batch), YOLO 1080p det-batch 4, FaceNet fp32 batch 128, ViT-L batch 8 and 128.
    Inputs are regenerated from seeds on the GPU box (synth.make_frames, numpy PCG64)."""
    import hashlib
    load_ref()
    out = {}
    m = importlib.import_module('ref_vtf.detectors.mtcnn')
    net = _load(m.MTCNN('cpu'), synth.make_params('mtcnn'))
    for name, n, seed, ms in (('mtcnn_b16_ms5', 16, 100, 5), ('mtcnn_b4_ms20', 4, 101, 20)):
        frames = synth.make_frames(n, seed=seed)
        with torch.inference_mode():
            res = net(list(frames), ms)
        out[name + '_counts'] = np.array([r.shape[0] for r in res], np.int64)
        out[name + '_boxes'] = np.concatenate(res).astype(np.float32)
        print(name, out[name + '_counts'])
    y = importlib.import_module('ref_vtf.detectors.yolo')
    ynet = _load(y.YOLOv3('cpu'), synth.make_params('yolo'))
    frames = synth.make_frames(4, 1080, 1920, seed=102)
    b, sc, resized = _yolo_ref(ynet, y, frames)
    out['yolo_1080_b4_counts'] = np.array([len(t) for t in sc], np.int64)
    out['yolo_1080_b4_boxes'] = np.concatenate(b)
    out['yolo_1080_b4_scores'] = np.concatenate(sc)
    out['yolo_1080_b4_resized_sha256'] = np.frombuffer(hashlib.sha256(np.stack(resized).tobytes()).digest(), np.uint8)
    print('yolo 1080p', out['yolo_1080_b4_counts'])
    f = importlib.import_module('ref_vtf.encoders.facenet')
    fnet = _load(f.InceptionResnetV1('cpu'), synth.make_params('facenet'))
    u8 = torch.from_numpy(_u8(103, (128, 3, 160, 160)))
    with torch.inference_mode():
        out['facenet_b128'] = fnet((u8.float() - 127.5) * (1 / 128)).numpy()
    v = importlib.import_module('ref_vtf.encoders.vit')
    vnet = _load(v.ViT('cpu', 128, 16, 1024, 24), synth.make_params('vit_l'))
    u8 = torch.from_numpy(_u8(104, (128, 3, 128, 128)))
    x = (u8.float() - 127.5) * np.float32(1 / 127.5)
    with torch.inference_mode():
        out['vit_l_b8'] = vnet(x[:8]).numpy()
        out['vit_l_b128'] = vnet(x).numpy()
    np.savez_compressed(os.path.join(HERE, 'shapes.npz'), **out)
    print('shapes', {k: v.shape for k, v in out.items()})


def gen_meta():
    """Host settings the goldens' bits depend on: torch's intra-op thread count (torch's CPU
    sigmoid splits a tensor into per-thread chunks: Sleef on vector steps, glibc on chunk tails,
    which rcnn.hip reproduces at VTF_TORCH_THREADS, default 8) and numpy's BLAS (the cosine
    dedupe's ssyrk order)."""
    import json
    import threadpoolctl
    blas = [(d.get('internal_api'), d.get('version'), d.get('architecture'), os.path.basename(d.get('filepath', '')))
            for d in threadpoolctl.threadpool_info() if d.get('user_api') == 'blas']
    meta = {'torch_threads': torch.get_num_threads(), 'numpy': np.__version__, 'blas': blas}
    with open(os.path.join(HERE, 'meta.json'), 'w') as f:
        json.dump(meta, f, indent=1)
    print('meta', meta)


def gen_b1():
    """BASELINE config 1's shape: MTCNN on 720p frames one at a time (det-batch 1) at the
    RealMTCNN default min_face_size 5 -- four single-frame calls (seeds 110..113); with one image
    per call every batched_nms segment is the whole call."""
    load_ref()
    m = importlib.import_module('ref_vtf.detectors.mtcnn')
    net = _load(m.MTCNN('cpu'), synth.make_params('mtcnn'))
    out = {'seeds': np.arange(110, 114)}
    for seed in out['seeds']:
        frames = synth.make_frames(1, seed=int(seed))
        with torch.inference_mode():
            res, ldm = net(list(frames), 5, return_landmarks=True)
        out['b1_%d_boxes' % seed] = res[0].astype(np.float32)
        out['b1_%d_landmarks' % seed] = ldm[0].astype(np.float32) if len(ldm) else np.zeros((0, 5, 2), np.float32)
        print('b1 seed', seed, res[0].shape)
    np.savez_compressed(os.path.join(HERE, 'b1.npz'), **out)


# MTCNN's float -> integer gates, per golden frame: the stage-1 / -2 / -3 score gates (p >= 0.6,
# s > 0.7: mtcnn.py:183, 215, 230), every batched_nms IoU against its threshold (0.5 / 0.7: 196,
# 205, 219) and the final IoM against 0.7 (242, 295-297).  A frame is flagged when one of its
# candidates sits within the device's tolerance of a gate: a score within FLAG_SCORE (5x the P/R/
# O-Net parity bar 2e-5), an IoU / IoM within FLAG_OVR of the threshold on refined boxes (stage 2
# / 3: box error <= 2e-3 px) or exactly ON it on stage 1's integer-grid boxes (bit-exact there).
FLAG_SCORE, FLAG_OVR, FLAG_OVR_EXACT = 1e-4, 1e-3, 1e-6
# stage-1 cells within NEAR_P of the p >= 0.6 gate (the PNet parity bar, test_pnet_level_vs_oracle)
# are recorded by key: the device's stage-1 set may differ from the reference's only there
NEAR_P = 2e-5
MTCNN_FLAG_RUNS = (('mtcnn_b16_ms5', 16, 100, 5), ('mtcnn_b4_ms20', 4, 101, 20),
                   ('b1_110', 1, 110, 5), ('b1_111', 1, 111, 5), ('b1_112', 1, 112, 5), ('b1_113', 1, 113, 5))


def _pair_margin(b, grp, thr, iom, plus1):
    """min |overlap - thr| over the same-group pairs (torchvision IoU: no +1, fp32 as nms_kernel;
    _nms_vectorized IoM: +1 widths, pairs with a positive intersection) per group id"""
    out = {}
    b = b.astype(np.float32)
    one = np.float32(1 if plus1 else 0)
    for gid in np.unique(grp):
        q = b[grp == gid]
        if len(q) < 2:
            continue
        best = np.inf
        area = (q[:, 2] - q[:, 0] + one) * (q[:, 3] - q[:, 1] + one)
        for i0 in range(0, len(q), 512):
            a = q[i0:i0 + 512, None]
            w = np.minimum(a[..., 2], q[None, :, 2]) - np.maximum(a[..., 0], q[None, :, 0]) + one
            h = np.minimum(a[..., 3], q[None, :, 3]) - np.maximum(a[..., 1], q[None, :, 1]) + one
            if iom:
                ok = (w > 0) & (h > 0)
                ov = (w * h) / np.minimum(area[i0:i0 + 512, None], area[None, :])
            else:
                w, h = np.maximum(w, 0), np.maximum(h, 0)
                inter = w * h
                ov = inter / ((area[i0:i0 + 512, None] + area[None, :]) - inter)
                ok = np.ones_like(ov, bool)
            ii = np.arange(i0, min(i0 + 512, len(q)))[:, None] < np.arange(len(q))[None, :]  # i < j pairs
            m = np.abs(ov.astype(np.float64) - thr)[ok & ii]
            if m.size:
                best = min(best, float(m.min()))
        out[int(gid)] = best
    return out


def gen_mtcnn_flags():
    """Near-threshold report of the MTCNN goldens (shapes.npz b16 / b4, b1.npz): the reference's
    forward on the same frames with its gates instrumented (wrappers around PNet / RNet / ONet,
    the candidate crops, torchvision.ops.batched_nms and _nms_vectorized record every decision's
    distance to its threshold per frame).  Saved per run: the flagged frames and each frame's
    smallest score / IoU / IoM margins; the GPU tests assert those frames' rows (all frames are
    asserted; the flagged ones are the ones a less precise kernel would lose first)."""
    load_ref()
    m = importlib.import_module('ref_vtf.detectors.mtcnn')
    net = _load(m.MTCNN('cpu'), synth.make_params('mtcnn'))
    ops = sys.modules['torchvision.ops']
    out = {}
    for name, n, seed, ms in MTCNN_FLAG_RUNS:
        rec = {'score': np.full(n, np.inf), 'iou': np.full(n, np.inf), 'iom': np.full(n, np.inf)}
        exact_iou = [True]  # stage-1 calls (integer-grid boxes) until the first RNet call
        cand_img = []
        ev = []  # the gates' integer outcomes in call order: (stage event, count)
        s1_keys, s1_near, s1_near_p = [], [], []

        def note(kind, img, marg):
            for i, v in zip(img, marg):
                rec[kind][int(i)] = min(rec[kind][int(i)], float(v))

        pnet_f, rnet_f, onet_f = net.pnet.forward, net.rnet.forward, net.onet.forward
        crop_f, nms_v, bnms = net._get_cropped_candidates, net._nms_vectorized, ops.batched_nms

        def pnet(x):
            reg, prob = pnet_f(x)
            d = np.abs(prob.numpy().astype(np.float64) - 0.6).reshape(prob.shape[0], -1).min(1)
            note('score', range(prob.shape[0]), d)
            ev.append(('mask', int((prob >= 0.6).sum())))
            lvl = sum(1 for e in ev if e[0] == 'mask') - 1
            pn = prob.numpy()
            lin = np.arange(pn.size, dtype=np.uint64).reshape(pn.shape)  # (b * ph + y) * pw + x
            s1_keys.append((np.uint64(lvl) << np.uint64(32)) | lin[pn >= 0.6])
            near = np.abs(pn.astype(np.float64) - 0.6) < NEAR_P
            s1_near.append((np.uint64(lvl) << np.uint64(32)) | lin[near])
            s1_near_p.append(pn[near])
            return reg, prob

        def crops(x, imgidx, boxes, size):
            exact_iou[0] = False
            cand_img.append(imgidx.numpy().copy())
            ev.append(('crops', int(imgidx.shape[0])))
            return crop_f(x, imgidx, boxes, size)

        def scored(f):
            def g(x):
                r = f(x)
                s_ = r[-1].numpy().astype(np.float64)
                note('score', cand_img[-1], np.abs(s_ - 0.7))
                ev.append(('pass', int((r[-1] > 0.7).sum())))
                return r
            return g

        def batched(boxes, scores, idxs, thr):
            for gid, v in _pair_margin(boxes.numpy(), idxs.numpy(), thr, False, False).items():
                if not exact_iou[0] or v <= FLAG_OVR_EXACT:
                    rec['iou'][gid] = min(rec['iou'][gid], v)
            k = bnms(boxes, scores, idxs, thr)
            ev.append(('nms', int(k.shape[0])))
            return k

        def vect(boxes, scores, classes, thresh, method, chain_suppression=True):
            for gid, v in _pair_margin(boxes.numpy(), classes.numpy(), thresh, True, True).items():
                rec['iom'][gid] = min(rec['iom'][gid], v)
            k = nms_v(boxes, scores, classes, thresh, method, chain_suppression)
            ev.append(('iom', int(k.shape[0])))
            return k

        net.pnet.forward, net.rnet.forward, net.onet.forward = pnet, scored(rnet_f), scored(onet_f)
        net._get_cropped_candidates, net._nms_vectorized, ops.batched_nms = crops, vect, batched
        try:
            with torch.inference_mode():
                res = net(list(synth.make_frames(n, seed=seed)), ms)
        finally:
            del net.pnet.forward, net.rnet.forward, net.onet.forward, net._get_cropped_candidates, net._nms_vectorized
            ops.batched_nms = bnms
        flagged = [f for f in range(n) if rec['score'][f] < FLAG_SCORE or rec['iou'][f] < FLAG_OVR
                   or rec['iom'][f] < FLAG_OVR]
        out[name + '_flagged'] = np.array(flagged, np.int64)
        out[name + '_counts'] = np.array([r.shape[0] for r in res], np.int64)
        # the device's stage counters (vtf_mtcnn_stats 1..7): stage-1 cells through the gate, kept
        # by the per-level NMS, by the cross-level NMS; RNet passes, kept by its NMS; ONet passes;
        # kept by the IoM NMS
        c1 = ev.index(next(e for e in ev if e[0] == 'crops'))
        nms1 = [v for k_, v in ev[:c1] if k_ == 'nms']
        rest = ev[c1:]
        st = [sum(v for k_, v in ev[:c1] if k_ == 'mask'), sum(nms1[:-1]), nms1[-1],
              [v for k_, v in rest if k_ == 'pass'][0], [v for k_, v in rest if k_ == 'nms'][0],
              [v for k_, v in rest if k_ == 'pass'][1], [v for k_, v in rest if k_ == 'iom'][0]]
        out[name + '_stage_counts'] = np.array(st, np.int64)
        out[name + '_s1_keys'] = np.concatenate(s1_keys)
        out[name + '_s1_near_keys'] = np.concatenate(s1_near)
        out[name + '_s1_near_p'] = np.concatenate(s1_near_p).astype(np.float32)
        for k in ('score', 'iou', 'iom'):
            out[name + '_margin_' + k] = rec[k]
        print(name, 'stage counts', st, 'flagged', flagged, 'min margins score %.3g iou %.3g iom %.3g'
              % (rec['score'].min(), rec['iou'].min(), rec['iom'].min()), flush=True)
    out['thresholds'] = np.array([FLAG_SCORE, FLAG_OVR, FLAG_OVR_EXACT, NEAR_P])
    np.savez_compressed(os.path.join(HERE, 'mtcnn_flags.npz'), **out)


# BASELINE config 5 chain: YOLO on 1080p frames -> box filter/adjust -> ViT-L on the crops ->
# cosine dedupe -> KMeans k=2..16 + scores; bench settings of the box filter
# (frames = synth.make_frame_sets(sets, per_set, 1080, 1920, seed, faces_per_frame): 128 frames)
CHAIN = dict(sets=16, per_set=8, faces_per_frame=12, det_batch=8, seed=600, mscore=0.4, msize=50, mborder=5,
             scale=(1.5, 1.5, 2.2, 1.2), square=True)


def _sk_kmeans_sweep(X, ks, threads):
    """cluster_faces' KMeans calls (grouping.py:99-101) with sklearn's OpenMP pool limited to
    `threads` (its n_threads = _openmp_effective_n_threads() at fit time)."""
    import sklearn.cluster
    from threadpoolctl import threadpool_limits
    with threadpool_limits(limits=threads, user_api='openmp'):
        return np.stack([sklearn.cluster.KMeans(n_clusters=k, random_state=0, n_init='auto').fit(X).labels_
                         for k in ks]).astype(np.int32)


def gen_chain():
    """Config-5 chain with the reference's own modules end to end (detector, detection.py box
    logic, ViT, dupes.remove_dupes_overall, sklearn KMeans/scores as cluster_faces calls them);
    cv2's resizes are the build's INTER_LINEAR restatement (parity-unpinned step)."""
    import json
    import sklearn.cluster
    import sklearn.metrics
    load_ref()
    sys.path.insert(0, ROOT)
    from oracle.facenet import resize_linear_u8
    c = CHAIN
    y = importlib.import_module('ref_vtf.detectors.yolo')
    det = importlib.import_module('ref_vtf.detection')
    dupes = importlib.import_module('ref_vtf.dupes')
    v = importlib.import_module('ref_vtf.encoders.vit')
    ynet = _load(y.YOLOv3('cpu'), synth.make_params('yolo'))
    vnet = _load(v.ViT('cpu', 128, 16, 1024, 24), synth.make_params('vit_l'))
    frames = synth.make_frame_sets(c['sets'], c['per_set'], 1080, 1920, c['seed'], c['faces_per_frame'])
    rects, margins, raw, flagged = [], [], [], []
    sp = ('', '', None, False, False, False)
    for j in range(0, len(frames), c['det_batch']):
        fb = frames[j:j + c['det_batch']]
        b, sc, _ = _yolo_ref(ynet, y, fb)
        for i, (bi, si) in enumerate(zip(b, sc)):
            rows = np.concatenate([bi, si[:, None]], 1)
            raw.append(rows)
            kept = det.filter_boxes(rows, (1080, 1920), c['mscore'], c['msize'], c['mborder'], sp, None, 0)
            adj = det.adjust_boxes(kept, (1080, 1920), c['scale'], c['square'])
            rects.extend((j + i, x1, y1, x2, y2) for (x1, y1, x2, y2, _) in adj)
            # fp32 re-association on the GPU can flip a floor/ceil only for a coordinate within a
            # few ulp of an integer, and the score gate only for a score within noise of
            # min_score: record both margins over the boxes the score gate could pass, and flag
            # the frames where one is inside the detector's parity tolerance
            live = si >= c['mscore'] - 1e-3
            if live.any():
                cm = np.abs(bi[live] - np.round(bi[live])).min()
                sm = np.abs(si - c['mscore']).min()
                margins.append(min(cm, sm))
                if cm < 2e-3 or sm < 1e-4:
                    flagged.append(j + i)
    rects = np.array(rects, np.int32)
    blobs = []
    for f, x1, y1, x2, y2 in rects:
        r = resize_linear_u8(frames[f, y1:y2, x1:x2], 128)[:, :, ::-1].transpose(2, 0, 1)
        blobs.append((torch.from_numpy(np.ascontiguousarray(r)).float() - 127.5) * np.float32(1 / 127.5))
    with torch.inference_mode():
        X = np.concatenate([vnet(torch.stack(blobs[i:i + 64])).numpy() for i in range(0, len(blobs), 64)])
    names = ['f%05d.jpg' % i for i in range(len(X))]
    with tempfile.TemporaryDirectory() as td:
        os.makedirs(os.path.join(td, 'faces'))
        for n in names:
            open(os.path.join(td, 'faces', n), 'w').close()
        Xk, goods = dupes.remove_dupes_overall(X.copy(), names, ('enc', 0.25, False, td))
    Dm = sklearn.metrics.pairwise.cosine_distances(X)
    Dm += (1 - np.tri(len(X), k=-1).astype(Dm.dtype)) * 10000
    # main.py:72-77: the sweep clusters the DEDUPED embeddings
    ks = [k for k in range(2, 17) if k <= len(Xk)]
    labels = _sk_kmeans_sweep(Xk, ks, 1)
    labels_mt = _sk_kmeans_sweep(Xk, ks, os.cpu_count())
    scores = [(sklearn.metrics.silhouette_score(Xk, lb), sklearn.metrics.calinski_harabasz_score(Xk, lb),
               sklearn.metrics.davies_bouldin_score(Xk, lb)) for lb in labels]
    out = dict(params_json=np.array(json.dumps(c)), rects=rects, X=X,
               dedupe_keep=np.array([int(n[1:6]) for n in goods], np.int64), dedupe_mins=Dm.min(1),
               dedupe_inds=Dm.argmin(1), k=np.array(ks), labels=labels, labels_mt=labels_mt,
               mt_threads=np.array(os.cpu_count()), scores=np.array(scores, np.float64),
               min_int_margin=np.array(min(margins)), flagged_frames=np.array(flagged, np.int64))
    np.savez_compressed(os.path.join(HERE, 'chain.npz'), **out)
    print('chain faces', len(X), 'kept after dedupe', len(goods), 'min |coord - round| %.4g' % min(margins),
          'flagged frames', flagged,
          'best k', ks[int(np.argmax([s[0] for s in scores]))],
          'sklearn 1 vs %d threads: rows differing per k' % os.cpu_count(), (labels != labels_mt).sum(1).tolist())


# BASELINE config 4's chain at N >= 10k: ViT-L/16 on 10,368 face crops (the blobs of 864 720p
# synthetic frames, 12 per frame: synth.make_frame_sets / face_rects; config 4's pre-cropped
# synth.make_crops patches of one background are near-duplicates of each other under the
# synthetic ViT-L -- the dedupe keeps 7 of 10,240 -- so they cannot exercise the sweep) ->
# remove_dupes_overall('enc') -> cluster_faces' KMeans sweep k = 2..16 + scores on the kept rows
C4CHAIN = dict(sets=54, per_set=16, faces_per_frame=12, seed=4100, thr=0.25, ks=list(range(2, 17)), sample=64)


def gen_c4chain():
    """Config-4-shaped grouping chain at N >= 10k with the reference's own ViT-L (AnimeVIT's blob
    restated: INTER_LINEAR to 128, parity-unpinned step) and dupes.remove_dupes_overall, then
    sklearn's KMeans / scores as cluster_faces calls them (1 OpenMP thread, and every core).
    Stored: a hash of the frames, the crop rectangles, every `sample`-th embedding row (the
    encoder's 1e-4 check), the dedupe result, int8 labels and the scores.  `perturbed_rows`:
    rows whose label moves when the kept X gets N(0, 1e-5) noise (the sweep's sensitivity at
    the encoder's tolerance; the device test reports its own)."""
    import hashlib
    import json
    import sklearn.metrics
    load_ref()
    sys.path.insert(0, ROOT)
    from oracle.facenet import resize_linear_u8
    c = C4CHAIN
    v = importlib.import_module('ref_vtf.encoders.vit')
    dupes = importlib.import_module('ref_vtf.dupes')
    vnet = _load(v.ViT('cpu', 128, 16, 1024, 24), synth.make_params('vit_l'))
    frames, faces = synth.make_frame_sets(c['sets'], c['per_set'], 720, 1280, c['seed'], c['faces_per_frame'],
                                          return_faces=True)
    rects = synth.face_rects(faces, 720, 1280)
    X = []
    for i in range(0, len(rects), 64):
        blobs = [(torch.from_numpy(np.ascontiguousarray(resize_linear_u8(frames[f, y1:y2, x1:x2], 128)[:, :, ::-1]
                                                        .transpose(2, 0, 1))).float() - 127.5) * np.float32(1 / 127.5)
                 for f, x1, y1, x2, y2 in rects[i:i + 64]]
        with torch.inference_mode():
            X.append(vnet(torch.stack(blobs)).numpy())
        if i % 1024 == 0:
            print('c4chain: encoded', i, flush=True)
    X = np.concatenate(X)
    names = ['f%05d.jpg' % i for i in range(len(X))]
    with tempfile.TemporaryDirectory() as td:
        os.makedirs(os.path.join(td, 'faces'))
        for n in names:
            open(os.path.join(td, 'faces', n), 'w').close()
        Xk, goods = dupes.remove_dupes_overall(X.copy(), names, ('enc', c['thr'], False, td))
    keep = np.array([int(n[1:6]) for n in goods], np.int64)
    ks = [k for k in c['ks'] if k < len(Xk)]
    labels = _sk_kmeans_sweep(Xk, ks, 1)
    labels_mt = _sk_kmeans_sweep(Xk, ks, os.cpu_count())
    scores = [(sklearn.metrics.silhouette_score(Xk, lb), sklearn.metrics.calinski_harabasz_score(Xk, lb),
               sklearn.metrics.davies_bouldin_score(Xk, lb)) for lb in labels]
    rng = np.random.default_rng(0)
    Xp = (Xk + rng.normal(0, 1e-5, Xk.shape)).astype(np.float32)
    pert = (_sk_kmeans_sweep(Xp, ks, 1) != labels).sum(1)
    np.savez_compressed(os.path.join(HERE, 'c4chain.npz'), params_json=np.array(json.dumps(c)),
                        frames_sha256=np.frombuffer(hashlib.sha256(frames.tobytes()).digest(), np.uint8),
                        rects=rects, X_sample=X[::c['sample']], dedupe_keep=keep.astype(np.int32), k=np.array(ks),
                        labels=labels.astype(np.int8), labels_mt=labels_mt.astype(np.int8),
                        mt_threads=np.array(os.cpu_count()), scores=np.array(scores, np.float64),
                        perturbed_rows=pert.astype(np.int64))
    print('c4chain: N', len(X), 'kept', len(keep), 'best k', ks[int(np.argmax([s[0] for s in scores]))],
          'sklearn 1 vs %d threads: rows differing per k' % os.cpu_count(), (labels != labels_mt).sum(1).tolist(),
          'rows moved by 1e-5 noise per k', pert.tolist())


C3 = dict(frames=32, seed=110, mscore=0.4, msize=50, mborder=5, scale=(1.5, 1.5, 2.2, 1.2), square=True)


def gen_c3():
    """BASELINE config 3's shapes end to end: YOLOv3 on one det-batch of 32 synthetic 720p
    frames -> the reference's filter_boxes / adjust_boxes (bench settings = reference defaults)
    -> FaceNet on the crops (blobFromImages restated: INTER_LINEAR 160x160, parity-unpinned
    step).  Reference modules throughout; frames flagged where a box coordinate lies within
    2e-3 px of an integer or a score within 1e-4 of min_score (as gen_chain)."""
    import json
    load_ref()
    sys.path.insert(0, ROOT)
    from oracle.facenet import resize_linear_u8
    c = C3
    y = importlib.import_module('ref_vtf.detectors.yolo')
    det = importlib.import_module('ref_vtf.detection')
    f = importlib.import_module('ref_vtf.encoders.facenet')
    ynet = _load(y.YOLOv3('cpu'), synth.make_params('yolo'))
    fnet = _load(f.InceptionResnetV1('cpu'), synth.make_params('facenet'))
    frames = synth.make_frames(c['frames'], seed=c['seed'])
    b, sc, _ = _yolo_ref(ynet, y, frames)
    rects, flagged, counts, boxes, scores = [], [], [], [], []
    sp = ('', '', None, False, False, False)
    for i, (bi, si) in enumerate(zip(b, sc)):
        rows = np.concatenate([bi, si[:, None]], 1)
        counts.append(len(rows))
        boxes.append(bi)
        scores.append(si)
        kept = det.filter_boxes(rows, (720, 1280), c['mscore'], c['msize'], c['mborder'], sp, None, 0)
        adj = det.adjust_boxes(kept, (720, 1280), c['scale'], c['square'])
        rects.extend((i, x1, y1, x2, y2) for (x1, y1, x2, y2, _) in adj)
        live = si >= c['mscore'] - 1e-3
        if live.any() and (np.abs(bi[live] - np.round(bi[live])).min() < 2e-3 or np.abs(si - c['mscore']).min() < 1e-4):
            flagged.append(i)
    rects = np.array(rects, np.int32).reshape(-1, 5)
    blobs = []
    for fi, x1, y1, x2, y2 in rects:
        r = resize_linear_u8(frames[fi, y1:y2, x1:x2], 160)[:, :, ::-1].transpose(2, 0, 1)
        blobs.append((torch.from_numpy(np.ascontiguousarray(r)).float() - 127.5) * np.float32(1 / 128))
    with torch.inference_mode():
        emb = fnet(torch.stack(blobs)).numpy() if blobs else np.zeros((0, 512), np.float32)
    np.savez_compressed(os.path.join(HERE, 'c3.npz'), params_json=np.array(json.dumps(c)),
                        counts=np.array(counts, np.int64), boxes=np.concatenate(boxes), scores=np.concatenate(scores),
                        rects=rects, emb=emb, flagged_frames=np.array(flagged, np.int64))
    print('c3: detections', sum(counts), 'crops', len(rects), 'flagged frames', flagged)


SCALE = dict(n=30000, seed=0, thr=0.25, ks=list(range(2, 17)))


def gen_scale():
    """Grouping at scale on realistic embeddings (BASELINE configs 4/5): N = 30k rows of
    synth.video_embeddings grown from the chain's ViT-L outputs (chain.npz X; regenerate this
    after gen_chain) -> the reference's embedding dedupe (dupes.py:60-65: cosine_distances +
    strict-lower-triangle min/argmin, threshold 0.25) -> on the kept rows (main.py:72-77)
    cluster_faces' KMeans sweep k = 2..16 and its three scores (grouping.py:97-107), sklearn
    with 1 OpenMP thread (deterministic) and with every core (its M-step reduces per-thread
    partial sums in lock order, so its last bits may depend on the thread count; rows where the
    two disagree are recorded).  Stored as a hash of X, the dedupe result and int8 labels."""
    import hashlib
    import sklearn.metrics
    c = SCALE
    X = synth.video_embeddings(np.load(os.path.join(HERE, 'chain.npz'))['X'], c['n'], seed=c['seed'])
    N = len(X)
    Dm = sklearn.metrics.pairwise.cosine_distances(X)
    mins = np.empty(N, np.float32)
    inds = np.empty(N, np.int64)
    # D += (1 - tri(N, k=-1)) * 10000 (dupes.py:62) one row block at a time: the same float32
    # elementwise adds as the reference's full-matrix statement, without its N x N float64 temps
    for i0 in range(0, N, 4096):
        blk = Dm[i0:i0 + 4096]
        blk += (1 - np.tri(N, k=-1)[i0:i0 + 4096].astype(blk.dtype)) * 10000
        mins[i0:i0 + 4096], inds[i0:i0 + 4096] = blk.min(1), blk.argmin(1)
    del Dm
    keep = np.nonzero(~(mins <= c['thr']))[0]
    Xk = X[keep]
    ks = [k for k in c['ks'] if k <= len(Xk)]
    labels = _sk_kmeans_sweep(Xk, ks, 1)
    labels_mt = _sk_kmeans_sweep(Xk, ks, os.cpu_count())
    scores = [(sklearn.metrics.silhouette_score(Xk, lb), sklearn.metrics.calinski_harabasz_score(Xk, lb),
               sklearn.metrics.davies_bouldin_score(Xk, lb)) for lb in labels]
    np.savez_compressed(os.path.join(HERE, 'scale.npz'), params_json=np.array(__import__('json').dumps(c)),
                        X_sha256=np.frombuffer(hashlib.sha256(X.tobytes()).digest(), np.uint8),
                        dedupe_mins=mins, dedupe_inds=inds.astype(np.int32), dedupe_keep=keep.astype(np.int32),
                        k=np.array(ks), labels=labels.astype(np.int8), labels_mt=labels_mt.astype(np.int8),
                        mt_threads=np.array(os.cpu_count()), scores=np.array(scores, np.float64))
    print('scale: N', N, 'kept', len(keep), 'best k', ks[int(np.argmax([s[0] for s in scores]))],
          'sklearn 1 vs %d threads: rows differing per k' % os.cpu_count(), (labels != labels_mt).sum(1).tolist())


def gen_iom():
    """MTCNN._nms_vectorized(..., 0.7, 'Min') (mtcnn.py:273-309) of the reference on crafted edge
    cases -- overlap chains (A~B~C with A, C apart: both B and C go), boxes touching on one pixel
    row (+1 widths make that an overlap), IoM exactly at the threshold, nested boxes, several
    classes -- and on random clustered boxes; distinct scores (the reference's argsort is
    unstable among ties)."""
    load_ref()
    m = importlib.import_module('ref_vtf.detectors.mtcnn')
    net = m.MTCNN('cpu')
    rng = np.random.default_rng(29)
    cases = {}
    crafted = np.array([
        [0, 0, 9, 9], [6, 0, 15, 9], [12, 0, 21, 9],            # chain: 0~1 (IoM 0.4?), 1~2
        [30, 30, 39, 39], [39, 30, 48, 39],                     # touch on one column (+1 -> inter 1x10)
        [50, 50, 59, 59], [50, 50, 59, 59],                     # identical
        [70, 70, 99, 99], [75, 75, 84, 84],                     # nested: IoM 1
        [100, 100, 109, 109], [103, 100, 112, 109],             # IoM = 7*10/100 = 0.7 exactly -> kept
        [120, 120, 129, 129], [122, 120, 131, 129],             # IoM 0.8
        [0, 0, 9, 9], [6, 0, 15, 9]], np.float32)               # same geometry, other class
    cls = np.array([0] * 13 + [1, 1], np.int64)
    sc = rng.permutation(len(crafted)).astype(np.float32) / len(crafted) + 0.01
    cases['crafted'] = (crafted, sc, cls)
    for name, n, spread in (('dense', 300, 60.0), ('sparse', 500, 600.0)):
        ctr = rng.uniform(0, spread, (n, 2)).astype(np.float32)
        wh = rng.uniform(4, 40, (n, 2)).astype(np.float32)
        b = np.concatenate([ctr, ctr + wh], 1)
        cases[name] = (b, rng.permutation(n).astype(np.float32) / n + 0.001, rng.integers(0, 3, n))
    out = {}
    for name, (b, sc, cls) in cases.items():
        with torch.inference_mode():
            keep = net._nms_vectorized(torch.from_numpy(b), torch.from_numpy(sc), torch.from_numpy(cls), 0.7, 'Min')
        out[name + '_boxes'], out[name + '_scores'], out[name + '_classes'] = b, sc, cls
        out[name + '_keep'] = keep.numpy()
        print('iom', name, len(b), '->', len(keep))
    np.savez_compressed(os.path.join(HERE, 'iom.npz'), **out)


# (H, W), mscore, msize, mborder, scale, square: the API / CLI / bench settings plus frames
# smaller than the scaled boxes (square overflow, side > other frame dimension, both
# orientations) and thresholds whose float32 rounding falls below the Python float (0.7)
BOX_CASES = [
    ((720, 1280), 0.4, 50, 5, (1.5, 1.5, 2.2, 1.2), True),
    ((720, 1280), 0.4, 0, 5, (1.5, 1.5, 2.2, 1.2), True),
    ((1080, 1920), 0.4, 50, 5, (1.5, 1.5, 2.2, 1.2), False),
    ((60, 100), 0.7, 0, 0, (2.0, 2.0, 3.0, 3.0), True),
    ((300, 120), 0.1, 3, 2, (1.25, 2.5, 1.75, 1.1), True),
    ((96, 96), 0.5, 1, 7.5, 2, True),
    ((200, 640), 0.0, 0, 0, (1, 1, 1, 1), True),
]


def box_rows(rng, H, W, n):
    """random detector rows (x1,y1,x2,y2,score) f32 over and around a HxW frame, with exact
    threshold scores, integer-valued corners, zero-size and out-of-frame boxes"""
    x1 = rng.uniform(-0.2 * W, 1.1 * W, n)
    y1 = rng.uniform(-0.2 * H, 1.1 * H, n)
    w = rng.uniform(0, 1.2 * max(H, W), n) * rng.choice([0.05, 0.3, 1.0], n)
    h = w * rng.uniform(0.3, 3.0, n)
    r = np.stack([x1, y1, x1 + w, y1 + h, rng.uniform(0, 1, n)], 1).astype(np.float32)
    k = n // 8
    r[:k, :4] = np.round(r[:k, :4])
    r[k:2 * k, 2] = r[k:2 * k, 0]
    r[2 * k:3 * k, 4] = rng.choice(np.array([0.4, 0.7, 0.5, 0.1, 0.0], np.float32), k)
    r[3 * k:4 * k, 4] = np.nextafter(rng.choice(np.array([0.4, 0.7], np.float32), k), np.float32(0))
    return r


def gen_boxes():
    """filter_boxes + adjust_boxes (detection.py:174-262) of the reference on random and
    edge-case boxes: inputs, and per case the kept (row, x1, y1, x2, y2)."""
    load_ref()
    det = importlib.import_module('ref_vtf.detection')
    rng = np.random.default_rng(23)
    out = {}
    save_params = ('', '', None, False, False, False)
    for ci, (sz, ms, mz, mb, sc, sq) in enumerate(BOX_CASES):
        rows = box_rows(rng, sz[0], sz[1], 1500)
        kept = det.filter_boxes(rows, sz, ms, mz, mb, save_params, None, 0)
        # filter_boxes returns rounded boxes; recover each one's row by its position among the
        # rows that pass (the reference keeps their order)
        adj = det.adjust_boxes(kept, sz, sc, sq)
        out['rows%d' % ci] = rows
        out['filtered%d' % ci] = np.array([b[:4] for b in kept], np.int64).reshape(-1, 4)
        out['filtered_score%d' % ci] = np.array([b[4] for b in kept], np.float32)
        out['adjusted%d' % ci] = np.array([b[:4] for b in adj], np.int64).reshape(-1, 4)
        print('boxes case', ci, sz, 'kept', len(kept), 'of', len(rows))
    import json
    out['cases_json'] = np.array(json.dumps(BOX_CASES))
    np.savez_compressed(os.path.join(HERE, 'boxes.npz'), **out)


# classify cases: (name, N, C, D, thr, seed) -- every numpy matmul order sklearn takes for
# X_n @ R_n.T (grouping_oracle.c): blocked sgemm (planted 10k x 8), small-matrix sgemm with an
# edge block (301 x 3), sgemv with 8 OpenBLAS threads (1003 x 1: 4x4 / 4x2 / 4x1 kernels per
# range), sgemv single thread (150 x 1), vector @ matrix (1 x 13), sdot (1 x 1)
CLASSIFY_CASES = [('planted', 10000, 8, 512, 0.9, 0), ('small', 301, 3, 768, 0.9, 1), ('gemv8', 1003, 1, 512, 0.9, 2),
                  ('gemv1', 150, 1, 1024, 0.9, 3), ('vecmat', 1, 13, 512, 0.9, 4), ('dot', 1, 1, 1024, 0.9, 5),
                  ('nothr', 500, 5, 512, None, 6)]


def gen_classify():
    """The reference's classify (grouping.py:50-66) on synth.classify_set data: the assigned
    indices (with 'other'), sklearn's distance matrix, and the log_classification.csv text."""
    import hashlib
    load_ref()
    grouping = importlib.import_module('ref_vtf.grouping')
    import sklearn.metrics
    out = {}
    for name, N, C, D, thr, seed in CLASSIFY_CASES:
        X, R = synth.classify_set(N, C, D, thr or 0.9, seed)
        classes = ['c%d' % i for i in range(C)]
        paths = ['/x/face_%05d.jpg' % i for i in range(N)]
        with tempfile.TemporaryDirectory() as td:
            os.makedirs(os.path.join(td, 'faces'))
            inds, classes = grouping.classify(X, R, classes, thr, True, paths, td)
            csv = open(os.path.join(td, 'faces', 'log_classification.csv')).read()
        out[name + '_inds'] = np.asarray(inds, np.int64)
        out[name + '_ncls'] = np.int64(len(classes))
        out[name + '_dist'] = sklearn.metrics.pairwise.cosine_distances(X, R)
        out[name + '_csv_sha'] = np.array(hashlib.sha256(csv.encode()).hexdigest())
        out[name + '_x_sha'] = np.array(hashlib.sha256(X.tobytes() + R.tobytes()).hexdigest())
    np.savez_compressed(os.path.join(HERE, 'classify.npz'), **out)
    print('classify', {k: v.shape for k, v in out.items()})


if __name__ == '__main__':
    which = sys.argv[1:] or ['mtcnn', 'facenet', 'vit', 'grouping', 'yolo', 'kmeans', 'rcnn', 'dupes', 'boxes', 'shapes', 'chain',
                             'scale', 'c3', 'iom', 'b1', 'classify', 'meta']
    for w in which:
        globals()['gen_' + w]()

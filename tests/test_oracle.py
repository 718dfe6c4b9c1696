"""CPU: pin the oracle (tests' CPU restatement) against golden vectors made from the
reference's own modules (tests/golden/make_golden.py)."""
import os
import sys

import numpy as np
import pytest
import torch
import torch.nn.functional as F

from conftest import GOLDEN


@pytest.fixture(scope='module')
def g():
    return np.load(os.path.join(GOLDEN, 'mtcnn.npz'))


@pytest.fixture(scope='module')
def params():
    from videotofaces import synth
    return synth.make_params('mtcnn')


def test_synth_weights_deterministic():
    from videotofaces import synth
    a = synth.hash_uniform('mtcnn:pnet.conv1.weight', 10)
    assert a.dtype == np.float32 and a.min() >= -1 and a.max() < 1
    np.testing.assert_array_equal(a, synth.hash_uniform('mtcnn:pnet.conv1.weight', 10))
    assert synth.pack(synth.make_params('mtcnn')).size == 495850


def test_oracle_nets_vs_golden(g, params):
    from oracle import mtcnn as om
    with torch.inference_mode():
        reg, prob = om.pnet(params, torch.from_numpy(g['pnet_in']))
        np.testing.assert_array_equal(reg.numpy(), g['pnet_reg'])
        np.testing.assert_array_equal(prob.numpy(), g['pnet_prob'])
        reg, prob = om.rnet(params, torch.from_numpy(g['rnet_in']))
        np.testing.assert_array_equal(reg.numpy(), g['rnet_reg'])
        np.testing.assert_array_equal(prob.numpy(), g['rnet_prob'])
        reg, lm, prob = om.onet(params, torch.from_numpy(g['onet_in']))
        np.testing.assert_array_equal(prob.numpy(), g['onet_prob'])
        np.testing.assert_array_equal(lm.numpy(), g['onet_lm'])


def test_oracle_pyramid_vs_golden(g):
    from oracle import mtcnn as om
    x = om.preprocess(list(g['pyr_frame']))
    scales, sizes = om.scale_pyramid(90, 160, 5)
    assert [tuple(s) for s in g['pyr_sizes']] == sizes[:4]
    for i, sz in enumerate(sizes[:4]):
        np.testing.assert_array_equal(F.adaptive_avg_pool2d(x, sz).numpy(), g['pyr_level%d' % i])


def test_oracle_adaptive_pool_restatement_bit_exact():
    # the kernel's bin-average rule: fp32 row-major sum, then /kh, then /kw
    rng = np.random.default_rng(0)
    u8 = rng.integers(0, 256, (1, 3, 37, 53)).astype(np.float32)
    x = torch.from_numpy((u8 - 127.5) / 128)
    for (oh, ow) in [(23, 31), (89, 120), (37, 53), (5, 7)]:
        ref = F.adaptive_avg_pool2d(x, (oh, ow))[0, 1].numpy()
        H, W = 37, 53
        for y in range(oh):
            y0, y1 = (y * H) // oh, -((-(y + 1) * H) // oh)
            for xx in range(ow):
                x0, x1 = (xx * W) // ow, -((-(xx + 1) * W) // ow)
                s = np.float32(0)
                for a in range(y0, y1):
                    for b in range(x0, x1):
                        s = np.float32(s + x[0, 1, a, b].numpy())
                v = np.float32(np.float32(s / np.float32(y1 - y0)) / np.float32(x1 - x0))
                assert v == ref[y, xx]


def test_oracle_e2e_small_frames_vs_golden(g, params):
    from oracle import mtcnn as om
    res = om.forward(params, list(g['small_frames']), minsize=5)
    k = 0
    for r, c in zip(res, g['small_ms5_counts']):
        np.testing.assert_array_equal(r, g['small_ms5_boxes'][k:k + c])
        k += c


def test_oracle_nms_c_core_vs_pure_torch():
    import sys
    sys.path.insert(0, GOLDEN)
    from oracle import nms as onms
    from make_golden import _tv_batched_nms
    rng = np.random.default_rng(1)
    for n, nimg in [(50, 2), (999, 3), (1200, 5)]:
        xy = rng.integers(0, 100, (n, 2)).astype(np.float32)
        b = torch.from_numpy(np.concatenate([xy, xy + rng.integers(3, 30, (n, 2))], 1).astype(np.float32))
        s = torch.from_numpy(rng.uniform(0, 1, n).astype(np.float32))
        i = torch.from_numpy(rng.integers(0, nimg, n))
        assert onms.batched_nms(b, s, i, 0.5).tolist() == _tv_batched_nms(b, s, i, 0.5).tolist()


def test_oracle_facenet_vs_golden():
    from videotofaces import synth
    from oracle.facenet import inception_resnet_v1
    gf = np.load(os.path.join(GOLDEN, 'facenet.npz'))
    x = (torch.from_numpy(gf['u8']).float() - 127.5) * (1 / 128)
    y = inception_resnet_v1(synth.make_params('facenet'), x).numpy()
    np.testing.assert_allclose(y, gf['emb'], atol=1e-6, rtol=0)


def _skylakex_blas():
    import threadpoolctl
    return any(d.get('internal_api') == 'openblas' and d.get('architecture') == 'SkylakeX'
               and 'numpy' in d.get('filepath', '') for d in threadpoolctl.threadpool_info())


@pytest.mark.parametrize('N,D', [(200, 512), (150, 1024), (120, 768), (100, 1000), (90, 200)])
def test_cosine_restatement_vs_sklearn(N, D):
    """oracle/grouping_oracle.c == sklearn cosine_distances bit for bit on every matrix entry
    (the orders were measured on numpy's OpenBLAS SkylakeX kernels: the comparison runs only
    where sklearn runs on those kernels; the goldens pin the same bits everywhere else)."""
    if not _skylakex_blas():
        pytest.skip('numpy BLAS is not OpenBLAS SkylakeX: sklearn bits differ from the pinned ones')
    from oracle import grouping as og
    rng = np.random.default_rng(D)
    X = rng.normal(0, 1, (N, D)).astype(np.float32)
    X[N // 2:N // 2 + 5] = X[3:8] + np.float32(1e-3)
    X[1] = 0
    ref = og.cosine_lower_sklearn(X)
    got = og.cosine_lower(X)
    np.testing.assert_array_equal(got, ref)
    mins, inds = og.cosine_dedupe(X)
    np.testing.assert_array_equal(mins, ref.min(1))
    np.testing.assert_array_equal(inds, ref.argmin(1))


def _openblas_threads():
    import threadpoolctl
    return [d.get('num_threads') for d in threadpoolctl.threadpool_info()
            if d.get('internal_api') == 'openblas' and 'numpy' in d.get('filepath', '')]


@pytest.mark.parametrize('N,C,D', [(10000, 8, 512), (600, 3, 512), (301, 3, 768), (37, 5, 1024), (2, 2, 512),
                                   (1003, 1, 512), (900, 1, 512), (899, 1, 512), (451, 1, 1024), (150, 1, 1024),
                                   (7, 1, 768), (1, 13, 512), (1, 5, 1024), (1, 1, 512), (1, 1, 1024)])
def test_classify_restatement_vs_sklearn(N, C, D):
    """oracle/grouping_oracle.c == sklearn cosine_distances(X, R) bit for bit for every matmul
    form sklearn reaches (blocked / small sgemm, sgemv's three kernels and its 8-thread split,
    sdot); the orders were measured on numpy's OpenBLAS SkylakeX kernels with 8 threads."""
    if not _skylakex_blas() or _openblas_threads() != [8]:
        pytest.skip('numpy BLAS is not 8-thread OpenBLAS SkylakeX: sklearn bits differ from the pinned ones')
    import sklearn.metrics
    from oracle import grouping as og
    from videotofaces import synth
    X, R = synth.classify_set(N, C, D, 0.9, seed=N + C + D)
    np.testing.assert_array_equal(og.classify_distances_exact(X, R), sklearn.metrics.pairwise.cosine_distances(X, R))


def test_oracle_classify_vs_golden():
    """the pinned restatement reproduces the reference's classify goldens (any host CPU)"""
    import hashlib
    from oracle import grouping as og
    from videotofaces import synth
    sys.path.insert(0, GOLDEN)
    from make_golden import CLASSIFY_CASES
    g = np.load(os.path.join(GOLDEN, 'classify.npz'))
    for name, N, C, D, thr, seed in CLASSIFY_CASES:
        X, R = synth.classify_set(N, C, D, thr or 0.9, seed)
        assert hashlib.sha256(X.tobytes() + R.tobytes()).hexdigest() == str(g[name + '_x_sha'])
        dist = og.classify_distances_exact(X, R)
        np.testing.assert_array_equal(dist, g[name + '_dist'])
        inds = dist.argmin(1)
        if thr:
            inds[dist.min(1) >= thr] = C
        np.testing.assert_array_equal(inds, g[name + '_inds'])


def test_oracle_grouping_vs_golden():
    from oracle import grouping as og
    gg = np.load(os.path.join(GOLDEN, 'grouping.npz'))
    mins, inds = og.cosine_dedupe(gg['X'])
    np.testing.assert_array_equal(mins, gg['dedupe_mins'])
    np.testing.assert_array_equal(inds, gg['dedupe_inds'])
    np.testing.assert_array_equal(np.nonzero(~(mins <= 0.25))[0], gg['dedupe_keep'])


def test_oracle_vit_vs_golden():
    from videotofaces import synth
    from oracle.vit import vit
    gv = np.load(os.path.join(GOLDEN, 'vit.npz'))
    x = (torch.from_numpy(gv['u8']).float() - 127.5) * np.float32(1 / 127.5)
    y = vit(synth.make_params('vit_b'), x, 768, 12).numpy()
    np.testing.assert_allclose(y, gv['vit_b'], atol=1e-5, rtol=0)


def test_oracle_yolo_vs_golden():
    """oracle/yolo.py (preprocess from the stored resized images, net, priors, postprocess,
    scale_boxes) against the reference YOLOv3 modules' outputs on the same synthetic weights."""
    from oracle import yolo as oy
    from videotofaces import synth
    from videotofaces.synth import make_frames
    gy = np.load(os.path.join(GOLDEN, 'yolo.npz'))
    fr = make_frames(2, seed=0)
    x, so, su = oy.preprocess(list(fr))
    assert su == [tuple(t) for t in gy['szu']] and so == [tuple(t) for t in gy['szo']]
    # the restated letterbox reproduces the golden input (both are the build's restatement;
    # pinned here so a change to either shows up)
    for i in range(2):
        h, w = gy['szu'][i]
        np.testing.assert_array_equal(
            (x[i, :, :h, :w] * 255).round().to(torch.uint8).permute(1, 2, 0).numpy()[..., ::-1], gy['resized'][i])
    p = synth.make_params('yolo')
    maps = oy.net(p, x)
    for i, m in enumerate(maps):
        np.testing.assert_allclose(m.numpy(), gy['map%d' % i], rtol=0, atol=1e-5 * np.abs(gy['map%d' % i]).max())
    with torch.inference_mode():
        b, s, c = oy.postprocess([torch.from_numpy(gy['map%d' % i]) for i in range(3)], oy.priors(x.shape[-2:]))
        sc = torch.tensor(so) / torch.tensor(su)
        sc = sc.flip(1).repeat(1, 2)
        b = [b[i] * sc[i] for i in range(len(b))]
    np.testing.assert_array_equal([len(t) for t in s], gy['counts'])
    np.testing.assert_array_equal(torch.cat(b).numpy(), gy['boxes'])
    np.testing.assert_array_equal(torch.cat(s).numpy(), gy['scores'])
    np.testing.assert_array_equal(torch.cat(c).numpy(), gy['classes'])


@pytest.fixture(scope='module')
def km():
    import hashlib
    from videotofaces import synth
    g = np.load(os.path.join(GOLDEN, 'kmeans.npz'))
    X = synth.planted_clusters()
    assert hashlib.sha256(X.tobytes()).digest() == g['X_sha256'].tobytes(), 'planted_clusters drifted'
    return g, X


def test_kmeans_host_control_flow_vs_sklearn(km):
    """videotofaces.kmeans.Grouper's sklearn control flow, driven by the numpy restatement of
    its device passes, reproduces sklearn's KMeans labels for k = 2..16 bit-exactly."""
    from oracle.kmeans import CpuGrouper
    g, X = km
    cg = CpuGrouper()
    prep = cg.prepare(X)
    for i, k in enumerate(g['k']):
        np.testing.assert_array_equal(cg.kmeans(X, int(k), prep=prep), g['labels'][i], err_msg='k=%d' % k)


def test_kmeans_host_control_flow_chain_deduped():
    """The same on the config-5 chain's deduped ViT-L embeddings (tests/golden/chain.npz, the
    reference flow main.py:72-77) against sklearn with one OpenMP thread."""
    from oracle.kmeans import CpuGrouper
    c = np.load(os.path.join(GOLDEN, 'chain.npz'))
    Xk = c['X'][c['dedupe_keep']]
    assert 0.3 < len(Xk) / len(c['X']) < 0.9, 'encoder calibration: dedupe keeps a real fraction'
    cg = CpuGrouper()
    prep = cg.prepare(Xk)
    for i, k in enumerate(c['k'][::3]):
        np.testing.assert_array_equal(cg.kmeans(Xk, int(k), prep=prep), c['labels'][3 * i], err_msg='k=%d' % k)


def test_video_embeddings_regenerate():
    """tests/golden/scale.npz's 30k embeddings regenerate bit-exactly from the chain's rows
    (synth.video_embeddings: elementwise float64 on numpy's PCG64 stream)."""
    import hashlib
    import json
    from videotofaces import synth
    g = np.load(os.path.join(GOLDEN, 'scale.npz'))
    c = json.loads(str(g['params_json']))
    X = synth.video_embeddings(np.load(os.path.join(GOLDEN, 'chain.npz'))['X'], c['n'], seed=c['seed'])
    assert hashlib.sha256(X.tobytes()).digest() == g['X_sha256'].tobytes()
    assert 0.3 < len(g['dedupe_keep']) / c['n'] < 0.9


def test_silhouette_restatement_vs_sklearn(km):
    from oracle.kmeans import silhouette_samples
    g, X = km
    sil = silhouette_samples(X, g['labels'][6])
    np.testing.assert_array_equal(sil, g['sil_k8'])
    assert float(np.mean(sil)) == g['scores'][6][0]


@pytest.fixture(scope='module')
def grc():
    return np.load(os.path.join(GOLDEN, 'rcnn.npz'))


def test_oracle_roi_align_vs_golden(grc):
    """oracle/rcnn.py's bin-vectorised torchvision roi_align restatement == the golden shim's
    sample-by-sample one (edge cases: outside the map, degenerate, large boxes)."""
    from oracle import rcnn as orc
    out = orc.roi_align(torch.from_numpy(grc['ra_fmap']), torch.from_numpy(grc['ra_rois']), 7, 0.25, True)
    np.testing.assert_array_equal(out.numpy(), grc['ra_out'])


def test_oracle_rcnn_small_heads_vs_golden(grc):
    from oracle import rcnn as orc
    from videotofaces import synth
    P = orc.params_t(synth.make_params('rcnn'))
    with torch.inference_mode():
        fm = orc.fpn(P, orc.body(P, torch.from_numpy(grc['small_x'])))
        for i, f in enumerate(fm):
            reg, log = orc.rpn_head(P, f)
            np.testing.assert_allclose(reg.numpy(), grc['small_reg%d' % i], rtol=0,
                                       atol=1e-5 * np.abs(grc['small_reg%d' % i]).max())
            np.testing.assert_allclose(log.numpy(), grc['small_log%d' % i], rtol=0,
                                       atol=1e-5 * np.abs(grc['small_log%d' % i]).max())


def test_oracle_rcnn_e2e_vs_golden(grc):
    """oracle/rcnn.py end to end (preprocess restated cv2 resize, ResNet50/FPN, RPN, RoIAlign,
    RoI head, NMS, scale_boxes) against the reference FasterRCNN on the same weights."""
    import hashlib
    from oracle import rcnn as orc
    from videotofaces import synth
    fr = synth.make_frames(2, seed=0)
    rs = [orc.resize_linear_u8_hw(f, orc.used_size(*f.shape[:2])) for f in fr]
    assert hashlib.sha256(np.stack(rs).tobytes()).digest() == grc['resized_sha256'].tobytes()
    b, s, c = orc.forward(synth.make_params('rcnn'), list(fr))
    np.testing.assert_array_equal([len(t) for t in s], grc['counts'])
    np.testing.assert_allclose(np.concatenate(b), grc['boxes'], rtol=0, atol=1e-3)
    np.testing.assert_allclose(np.concatenate(s), grc['scores'], rtol=0, atol=1e-5)


def test_oracle_hash_dedupe_vs_golden():
    """remove_dupes_overall('hash') distances (dupes.py:55-65): oracle == reference."""
    from oracle import dupes as od
    gd = np.load(os.path.join(GOLDEN, 'dupes.npz'))
    mins, inds = od.hamming_lower(gd['X'])
    np.testing.assert_array_equal(mins, gd['mins'])
    np.testing.assert_array_equal(inds, gd['inds'])
    np.testing.assert_array_equal(np.nonzero(~(mins <= 8))[0], gd['keep'])


def test_oracle_ahash_properties():
    """ahash restatement: identity at 8x8, 2x INTER_AREA path, hash = thumbnail > mean."""
    from oracle import dupes as od
    rng = np.random.default_rng(2)
    img = rng.integers(0, 256, (8, 8, 3)).astype(np.uint8)
    g = od.gray(img)
    np.testing.assert_array_equal(od.ahash(img), 1 * (g > g.mean()).flatten())
    big = np.repeat(np.repeat(img, 2, 0), 2, 1)
    np.testing.assert_array_equal(od.resize8(od.gray(big)), g)


def test_pack_hashes_roundtrip():
    from videotofaces.dupes import pack_hashes, unpack_hash
    rng = np.random.default_rng(3)
    H = rng.integers(0, 2, (5, 64))
    P = pack_hashes(H)
    assert P.dtype == np.uint64
    for h, p in zip(H, P):
        np.testing.assert_array_equal(unpack_hash(p), h)


@pytest.mark.parametrize('case', ['crafted', 'dense', 'sparse'])
def test_oracle_iom_chain_vs_reference(case):
    """oracle.mtcnn.nms_iom_chain (mtcnn.py:273-309 restated) vs the reference's own
    _nms_vectorized on edge cases (tests/golden/iom.npz)."""
    from oracle import mtcnn as om
    gi = np.load(os.path.join(GOLDEN, 'iom.npz'))
    keep = om.nms_iom_chain(torch.from_numpy(gi[case + '_boxes']), torch.from_numpy(gi[case + '_scores']),
                            torch.from_numpy(gi[case + '_classes']), 0.7)
    np.testing.assert_array_equal(np.asarray(keep), gi[case + '_keep'])


def test_golden_host_meta():
    """The goldens record the host settings their bits depend on (make_golden.py gen_meta): the
    device RPN reproduces torch's CPU sigmoid chunking at VTF_TORCH_THREADS (default 8) and the
    cosine dedupe the SkylakeX ssyrk order -- both must be what the goldens were made with."""
    import json
    meta = json.load(open(os.path.join(GOLDEN, 'meta.json')))
    assert meta['torch_threads'] == int(os.environ.get('VTF_TORCH_THREADS', '8'))
    assert any(b[0] == 'openblas' and b[2] == 'SkylakeX' for b in meta['blas'])

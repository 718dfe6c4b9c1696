"""GPU parity at the BENCHMARKED shapes (BASELINE configs 2-5), against golden vectors made by
the reference's own modules (tests/golden/make_golden.py gen_shapes / gen_chain):

* MTCNN 720p, det-batch 16 at min_face_size 5 (config 2), det-batch 4 at 20 (main.py:18's
  default batch) and det-batch 1 at 5 (config 1): batched_nms offsets depend on the batch composition (mtcnn.py:196,205,219);
* YOLOv3 on 1080p frames, det-batch 4 (configs 3/5 detector at the config-5 frame size);
* FaceNet fp32 at batch 128 and ViT-L at batch 8 and 128 (the multi-tile / split-K GEMM paths
  that run at enc-batch 128);
* the config-5 chain end to end: YOLO 1080p -> device box post-processing -> ViT-L on the device
  crops -> fused cosine dedupe -> KMeans k=2..16 + scores.

Tolerances: counts / crop rectangles / dedupe argmin and keep sets / KMeans labels exact;
detector boxes as the per-model tests (MTCNN 2e-3 px, YOLO 1e-2 px, scores 1e-4); embeddings
1e-4 (fp32 and split-fp16 operand modes); cosine minima 1e-5; scores rtol 1e-5.
"""
import json
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def g():
    return np.load(os.path.join(GOLDEN, 'shapes.npz'))


@pytest.fixture(scope='module')
def chain():
    return np.load(os.path.join(GOLDEN, 'chain.npz'))


def _u8(seed, shape):
    return np.random.default_rng(seed).integers(0, 256, shape, dtype=np.uint8)


@pytest.fixture(scope='module')
def mflags():
    return np.load(os.path.join(GOLDEN, 'mtcnn_flags.npz'))


def _mtcnn_gates(mflags, name, model, res, ref_rows):
    """Integer outcomes of every MTCNN gate vs the reference (make_golden.py gen_mtcnn_flags).
    Stage 1: the device's candidate set (cells with p >= 0.6, by key; recording enabled before the
    call) equals the reference's except on cells the reference puts within 2e-5 of the gate (the
    PNet parity bar) -- there the fp32 summation order decides, and the reference's own rounding is
    of that size; when the sets are equal, every later counter (kept by the per-level and
    cross-level NMS, RNet / ONet passes, kept by the stage-2 and the IoM NMS) is exact.  Then the
    golden's flagged frames (a score within 1e-4 of its gate, an IoU / IoM within 1e-3 of its
    threshold, or exactly on it for stage 1's integer boxes) row for row."""
    keys = model.stage1_keys()
    ref, near = mflags[name + '_s1_keys'], mflags[name + '_s1_near_keys']
    diff = np.setxor1d(keys, ref)
    assert np.isin(diff, near).all(), ('stage-1 candidates differ away from the gate', diff[~np.isin(diff, near)][:8])
    if diff.size == 0:
        np.testing.assert_array_equal(model.last_stats[1:8], mflags[name + '_stage_counts'], err_msg='stage counts')
    else:
        p = mflags[name + '_s1_near_p'][np.searchsorted(near, diff)]
        print('%s: %d stage-1 cell(s) on the other side of the gate, |p - 0.6| = %s' % (name, diff.size, np.abs(p.astype(np.float64) - 0.6)))
    fl = mflags[name + '_flagged']
    for f in fl:
        assert res[f].shape == ref_rows[f].shape, (name, f)
        np.testing.assert_allclose(res[f], ref_rows[f], rtol=1e-5, atol=2e-3, err_msg='flagged frame %d' % f)
    print('%s: stage counts %s (device %s); stage-1 cells within 2e-5 of the gate %d, differing %d; flagged frames '
          '%d of %d, smallest margins: score %.2g, IoU %.2g, IoM %.2g'
          % (name, mflags[name + '_stage_counts'].tolist(), model.last_stats[1:8].tolist(), near.size, diff.size, len(fl),
             len(res), mflags[name + '_margin_score'].min(), mflags[name + '_margin_iou'].min(), mflags[name + '_margin_iom'].min()))


@pytest.mark.parametrize('name,n,seed,ms', [('mtcnn_b16_ms5', 16, 100, 5), ('mtcnn_b4_ms20', 4, 101, 20)])
def test_mtcnn_benchmark_batches(g, mflags, name, n, seed, ms):
    from videotofaces import synth
    from videotofaces.detectors.mtcnn import MTCNN
    frames = synth.make_frames(n, seed=seed)
    m = MTCNN('cuda:0')
    m.stage1_keys(1)
    res = m(torch.from_numpy(frames).cuda(), ms)
    np.testing.assert_array_equal([r.shape[0] for r in res], g[name + '_counts'])
    np.testing.assert_allclose(np.concatenate(res), g[name + '_boxes'], rtol=1e-5, atol=2e-3)
    _mtcnn_gates(mflags, name, m, res, np.split(g[name + '_boxes'], np.cumsum(g[name + '_counts'])[:-1]))


def test_mtcnn_det_batch1_720p(mflags):
    """BASELINE config 1's shape: MTCNN on single 720p frames (det-batch 1, min_face_size 5),
    four calls, against the reference module (tests/golden/make_golden.py gen_b1): counts exact,
    boxes 2e-3 px, landmarks 2e-3 px, every gate's integer outcome (stage counters) exact."""
    from videotofaces import synth
    from videotofaces.detectors.mtcnn import MTCNN
    gb = np.load(os.path.join(GOLDEN, 'b1.npz'))
    m = MTCNN('cuda:0')
    m.stage1_keys(1)
    for seed in gb['seeds']:
        frames = synth.make_frames(1, seed=int(seed))
        res, ldm = m(torch.from_numpy(frames).cuda(), 5, return_landmarks=True)
        ref = gb['b1_%d_boxes' % seed]
        assert res[0].shape == ref.shape, (seed, res[0].shape, ref.shape)
        np.testing.assert_allclose(res[0], ref, rtol=1e-5, atol=2e-3)
        np.testing.assert_allclose(ldm[0], gb['b1_%d_landmarks' % seed], rtol=1e-5, atol=2e-3)
        _mtcnn_gates(mflags, 'b1_%d' % seed, m, res, [ref])


def test_mtcnn_b16_device_crops(g):
    """config 2's hand-off: detect_crops on det-batch 16 == the reference's boxes through the
    reference box logic (oracle/boxes.py, pinned by tests/golden/boxes.npz): every crop rectangle
    equal, no exemptions (the golden's box coordinates keep > 2e-3 px from every integer, so the
    device boxes' tolerance cannot move a floor / ceil: asserted too)."""
    from oracle.boxes import rows_to_crops
    from videotofaces import synth, _native as nat
    from videotofaces.detectors.mtcnn import MTCNN
    frames = synth.make_frames(16, seed=100)
    rows = np.split(g['mtcnn_b16_ms5_boxes'], np.cumsum(g['mtcnn_b16_ms5_counts'])[:-1])
    ref, src = rows_to_crops(rows, (720, 1280), 0.4, 0, 5, (1.5, 1.5, 2.2, 1.2), True)
    d, counts = MTCNN('cuda:0').detect_crops(torch.from_numpy(frames).cuda(), 5,
                                             nat.BoxParams.make(0.4, 0, 5, (1.5, 1.5, 2.2, 1.2), True))
    got = d.cpu().numpy()
    flat = np.concatenate(rows)
    start = np.concatenate([[0], np.cumsum(g['mtcnn_b16_ms5_counts'])[:-1]])
    near = (np.abs(flat[start[ref[:, 0]] + src, :4] - np.round(flat[start[ref[:, 0]] + src, :4])) < 2e-3).any(1)
    print('crops', len(ref), 'near-integer golden rows', int(near.sum()))
    assert not near.any()
    np.testing.assert_array_equal(got, ref)


def test_mtcnn_sat_layouts_bit_identical(g, monkeypatch):
    """The packed 8-byte SAT (default when every bin is under 8224 px) and the int3 SAT
    (VTF_SAT_PACK=0, the fallback for larger bins) give identical detections on config 2's
    det-batch: the box sums are exact integers either way (mtcnn_dev.hpp)."""
    from videotofaces import synth
    from videotofaces.detectors.mtcnn import MTCNN
    frames = torch.from_numpy(synth.make_frames(16, seed=100)).cuda()
    m = MTCNN('cuda:0')
    packed = m(frames, 5)
    monkeypatch.setenv('VTF_SAT_PACK', '0')
    wide = m(frames, 5)
    assert [r.shape[0] for r in packed] == [r.shape[0] for r in wide]
    for a, b in zip(packed, wide):
        np.testing.assert_array_equal(a, b)
    np.testing.assert_array_equal([r.shape[0] for r in packed], g['mtcnn_b16_ms5_counts'])


def test_mtcnn_strided_view_matches_contiguous():
    """A video_area-style view (rows and columns cropped in place: the frame base 9 bytes past a
    4-byte boundary) runs the block-per-row SAT pass, its contiguous copy the wave-per-row pass
    with LDS staging: identical detections either way."""
    from videotofaces import synth
    from videotofaces.detectors.mtcnn import MTCNN
    frames = torch.from_numpy(synth.make_frames(8, seed=7)).cuda()
    view = frames[:, 10:710, 3:1279]
    m = MTCNN('cuda:0')
    a = m(view, 5)
    b = m(view.contiguous(), 5)
    assert sum(r.shape[0] for r in a) > 0
    assert [r.shape[0] for r in a] == [r.shape[0] for r in b]
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)


@pytest.mark.parametrize('env', [{'VTF_PNET_PR': '0'}, {'VTF_PNET_X': '0', 'VTF_PNET_PR': '0'}, {'VTF_PNET_VR': '1'}])
def test_mtcnn_b16_pnet_variants(g, env, monkeypatch):
    """k_pnet's launch plans on config 2's det-batch against the same reference golden: the default
    (exact-levels variant + the PR variant on the levels precomputed as split pixels), the general
    variant instead of PR (VTF_PNET_PR=0), one general launch for every tile (VTF_PNET_X=0 too)
    and the vertical-reuse variants of both launches (VTF_PNET_VR=1: a continuing tile's shared
    pooled / conv2 rows reloaded from its workgroup's slot) -- counts exact, boxes 2e-3 px each;
    the plans read the same level values (bit-identical fills), so they also agree with each
    other to the same tolerance."""
    from videotofaces import synth
    from videotofaces.detectors.mtcnn import MTCNN
    frames = torch.from_numpy(synth.make_frames(16, seed=100)).cuda()
    m = MTCNN('cuda:0')
    base = m(frames, 5)
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    alt = m(frames, 5)
    for res in (base, alt):
        np.testing.assert_array_equal([r.shape[0] for r in res], g['mtcnn_b16_ms5_counts'])
        np.testing.assert_allclose(np.concatenate(res), g['mtcnn_b16_ms5_boxes'], rtol=1e-5, atol=2e-3)
    np.testing.assert_allclose(np.concatenate(alt), np.concatenate(base), rtol=1e-5, atol=2e-3)


def test_mtcnn_detect_crops_capacity_retry():
    """detect_crops with a crop capacity far below the kept count: the device box pass counts past
    the capacity without writing, the call reports VTF_E_CAPACITY with the needed size, and the
    retry (videotofaces._native.run_detect_crops) returns exactly the crops of a roomy call."""
    from videotofaces import synth, _native as nat
    from videotofaces.detectors.mtcnn import MTCNN
    frames = torch.from_numpy(synth.make_frames(16, seed=100)).cuda()
    m = MTCNN('cuda:0')
    bp = nat.BoxParams.make(0.4, 0, 5, (1.5, 1.5, 2.2, 1.2), True)
    ref, ref_counts = m.detect_crops(frames, 5, bp)
    assert ref.shape[0] > 2
    L = nat.lib()
    m._bind_stream()
    base, on_dev, B, H, W, fs, rs, keep = nat.frames_view(frames, m.device)
    calls = []

    def call(d, c, cap, n):
        calls.append(cap)
        return L.vtf_mtcnn_detect_crops(m._h, base, on_dev, B, H, W, fs, rs, 5.0, nat.ctypes.byref(bp), 0, d, c,
                                        cap, n)
    got, counts = nat.run_detect_crops(call, m.device, B, 1)
    assert calls[0] == 1 and len(calls) == 2 and calls[1] == ref.shape[0]
    np.testing.assert_array_equal(got.cpu().numpy(), ref.cpu().numpy())
    np.testing.assert_array_equal(counts, ref_counts)


@pytest.mark.parametrize('precision', ['fp32', 'x3'])
def test_yolo_1080p_b4(g, precision):
    from videotofaces import synth
    from videotofaces.detectors.yolo import YOLOv3
    frames = synth.make_frames(4, 1080, 1920, seed=102)
    b, s, c = YOLOv3('cuda:0', precision=precision)(torch.from_numpy(frames).cuda())
    np.testing.assert_array_equal([len(t) for t in s], g['yolo_1080_b4_counts'])
    np.testing.assert_allclose(np.concatenate(b), g['yolo_1080_b4_boxes'], rtol=1e-6, atol=1e-2)
    np.testing.assert_allclose(np.concatenate(s), g['yolo_1080_b4_scores'], rtol=1e-6, atol=1e-4)


@pytest.fixture(scope='module')
def c3():
    return np.load(os.path.join(GOLDEN, 'c3.npz'))


@pytest.mark.parametrize('precision', ['x3', 'fp32'])
def test_config3_det_batch32(c3, precision):
    """BASELINE config 3's det-batch: YOLOv3 on 32 720p frames in ONE call (the bench's tile /
    grid / split-K choices for B = 32) -> device box post-processing -> FaceNet on the device
    crops, against the reference modules (tests/golden/make_golden.py gen_c3): counts exact,
    boxes 1e-2 px, scores 1e-4; crop rectangles exact on every frame, including those the golden
    flags (a coordinate within 2e-3 px of an integer or a score within 1e-4 of min_score); FaceNet on
    the golden rectangles fp32 within 1e-4, bf16 (the config's encoder precision) cos >= 0.998."""
    import json
    from videotofaces import synth, _native as nat
    from videotofaces.detectors.yolo import YOLOv3
    from videotofaces.encoders.facenet import InceptionResnetV1
    c = json.loads(str(c3['params_json']))
    frames = torch.from_numpy(synth.make_frames(c['frames'], seed=c['seed'])).cuda()
    det = YOLOv3('cuda:0', precision=precision)
    b, s, _ = det(frames)
    np.testing.assert_array_equal([len(t) for t in s], c3['counts'])
    np.testing.assert_allclose(np.concatenate(b), c3['boxes'], rtol=1e-6, atol=1e-2)
    np.testing.assert_allclose(np.concatenate(s), c3['scores'], rtol=1e-6, atol=1e-4)
    d, _ = det.detect_crops(frames, nat.BoxParams.make(c['mscore'], c['msize'], c['mborder'], tuple(c['scale']),
                                                        c['square']))
    got, ref = d.cpu().numpy(), c3['rects']
    flagged = set(c3['flagged_frames'].tolist())
    # every frame, the flagged ones included (their outcome is reported first)
    same = [f for f in sorted(flagged) if np.array_equal(got[got[:, 0] == f], ref[ref[:, 0] == f])]
    print('c3 flagged frames %s: identical %s' % (sorted(flagged), same))
    for f in range(c['frames']):
        np.testing.assert_array_equal(got[got[:, 0] == f], ref[ref[:, 0] == f], err_msg='frame %d' % f)
    rects = torch.from_numpy(ref).cuda()
    emb = InceptionResnetV1('cuda:0', precision='fp32').encode_crops(frames, rects).cpu().numpy()
    np.testing.assert_allclose(emb, c3['emb'], rtol=0, atol=1e-4)
    bf = InceptionResnetV1('cuda:0', precision='bf16').encode_crops(frames, rects).cpu().numpy()
    cos = (bf * c3['emb']).sum(1) / np.linalg.norm(bf, axis=1)
    print('c3: %d detections, %d crops, flagged frames %s; FaceNet bf16 cos min %.6f'
          % (len(np.concatenate(s)), len(ref), sorted(flagged), cos.min()))
    # (bf16 is a perf mode, reported as drift; the calibrated BatchNorm centres the embedding,
    # so its relative bf16 error is larger than on the uncalibrated, collapsed one)
    assert cos.min() > 0.998


def test_facenet_fp32_batch128(g):
    from videotofaces.encoders.facenet import InceptionResnetV1
    x = (torch.from_numpy(_u8(103, (128, 3, 160, 160))).float() - 127.5) * (1 / 128)
    emb = InceptionResnetV1('cuda:0', precision='fp32')(x).cpu().numpy()
    np.testing.assert_allclose(emb, g['facenet_b128'], rtol=0, atol=1e-4)
    bf = InceptionResnetV1('cuda:0', precision='bf16')(x).cpu().numpy()
    cos = (bf * g['facenet_b128']).sum(1) / np.linalg.norm(bf, axis=1)
    print('facenet bf16 batch 128: cos min %.6f mean %.6f' % (cos.min(), cos.mean()))
    assert cos.min() > 0.999


@pytest.mark.parametrize('precision', ['fp32', 'f16x'])
def test_vit_l_batches(g, precision):
    from videotofaces import synth
    from videotofaces.encoders.vit import ViT
    m = ViT('cuda:0', synth.make_params('vit_l'), isL=True, precision=precision)
    x = (torch.from_numpy(_u8(104, (128, 3, 128, 128))).float() - 127.5) * np.float32(1 / 127.5)
    np.testing.assert_allclose(m(x[:8]).cpu().numpy(), g['vit_l_b8'], rtol=0, atol=1e-4)
    np.testing.assert_allclose(m(x).cpu().numpy(), g['vit_l_b128'], rtol=0, atol=1e-4)


@pytest.mark.parametrize('precision', ['fp32', 'f16x'])
def test_config5_chain(chain, precision):
    """Config 5 end to end on 128 1080p frames (488 faces): YOLO -> device box post-processing
    -> ViT-L on device crops -> fused cosine dedupe -> KMeans k=2..16 + scores on the DEDUPED
    rows (main.py:72-77).  Crop rectangles are exact on every frame, including the ones the
    golden flags (a box coordinate within 2e-3 px of an integer or a score within 1e-4 of
    min_score, where the detector's fp32 tolerance could decide a floor or a gate; the count of
    those that match is reported first); the encoder then runs on the
    golden rectangles, so the grouping half is checked on the reference's rows."""
    from videotofaces import synth, dupes
    from videotofaces.detection import detect_crops
    from videotofaces.detectors.yolo import YOLOv3
    from videotofaces.encoders.vit import ViT
    from videotofaces.grouping import cluster_sweep
    c = json.loads(str(chain['params_json']))
    frames_np = synth.make_frame_sets(c['sets'], c['per_set'], 1080, 1920, c['seed'], c['faces_per_frame'])
    frames = torch.from_numpy(frames_np).cuda()
    det = YOLOv3('cuda:0', precision='fp32')
    parts = []
    for j in range(0, len(frames), c['det_batch']):
        d, _ = detect_crops(det, frames[j:j + c['det_batch']], j, c['mscore'], c['msize'], c['mborder'],
                            tuple(c['scale']), c['square'])
        parts.append(d)
    got = torch.cat(parts).cpu().numpy()
    flagged = set(chain['flagged_frames'].tolist())
    same_flagged = sum(int(np.array_equal(got[got[:, 0] == f], chain['rects'][chain['rects'][:, 0] == f]))
                       for f in flagged)
    print('flagged frames %d, of which identical %d' % (len(flagged), same_flagged))
    for f in range(len(frames)):
        a, b = got[got[:, 0] == f], chain['rects'][chain['rects'][:, 0] == f]
        np.testing.assert_array_equal(a, b, err_msg='frame %d' % f)
    enc = ViT('cuda:0', synth.make_params('vit_l'), isL=True, precision=precision)
    X = enc.encode_crops(frames, torch.from_numpy(chain['rects']).cuda())
    np.testing.assert_allclose(X.cpu().numpy(), chain['X'], rtol=0, atol=1e-4)
    mins, inds = dupes.cosine_dedupe_device(torch.from_numpy(chain['X']).cuda())
    np.testing.assert_array_equal(mins, chain['dedupe_mins'])
    np.testing.assert_array_equal(inds, chain['dedupe_inds'])
    mins, inds = dupes.cosine_dedupe_device(X)  # on the device embeddings (within 1e-4)
    np.testing.assert_array_equal(np.nonzero(~(mins <= 0.25))[0], chain['dedupe_keep'])
    ks = [int(k) for k in chain['k']]
    # on the golden's own embeddings (bit-exact input) the labels equal sklearn's (1 OpenMP
    # thread; sklearn with every core agrees on these rows)
    Xk = chain['X'][chain['dedupe_keep']]
    assert np.array_equal(chain['labels'], chain['labels_mt'])
    labels, scores = cluster_sweep(Xk, ks, 0)
    for i, k in enumerate(ks):
        np.testing.assert_array_equal(labels[i], chain['labels'][i], err_msg='k=%d' % k)
    np.testing.assert_allclose(np.array([s[1:] for s in scores]), chain['scores'], rtol=1e-5)
    # the device embeddings (within 1e-4 of the golden's) -> the same labels for every k
    labels_dev, _ = cluster_sweep(X.cpu().numpy()[chain['dedupe_keep']], ks, 0)
    print('device embeddings: rows whose label differs per k',
          [int((a != b).sum()) for a, b in zip(labels_dev, chain['labels'])])
    for i, k in enumerate(ks):
        np.testing.assert_array_equal(labels_dev[i], chain['labels'][i], err_msg='device embeddings, k=%d' % k)


@pytest.mark.parametrize('precision', ['fp32', 'f16x'])
def test_config4_chain_10k(precision):
    """Config 4's encoder -> grouping chain at N = 10,368: ViT-L/16 on the device over the face
    crops of 864 synthetic 720p frames (regenerated here, hash-checked; the golden's crop
    rectangles) -> fused cosine dedupe -> KMeans k = 2..16 on the kept rows, against the
    reference's ViT-L + remove_dupes_overall + sklearn (make_golden.py gen_c4chain): sampled
    embeddings within 1e-4, the keep set and every k's labels exact on the DEVICE embeddings,
    silhouette / CH / DB within 1e-3."""
    import hashlib
    from videotofaces import synth, dupes
    from videotofaces.encoders.vit import ViT
    from videotofaces.grouping import cluster_sweep
    gc = np.load(os.path.join(GOLDEN, 'c4chain.npz'))
    c = json.loads(str(gc['params_json']))
    frames = synth.make_frame_sets(c['sets'], c['per_set'], 720, 1280, c['seed'], c['faces_per_frame'], threads=16)
    assert hashlib.sha256(frames.tobytes()).digest() == gc['frames_sha256'].tobytes()
    fd = torch.from_numpy(frames).cuda()
    rects = torch.from_numpy(gc['rects']).cuda()
    n = rects.shape[0]
    enc = ViT('cuda:0', synth.make_params('vit_l'), isL=True, precision=precision)
    X = torch.cat([enc.encode_crops(fd, rects[i:i + 128]) for i in range(0, n, 128)])
    Xh = X.cpu().numpy()
    np.testing.assert_allclose(Xh[::c['sample']], gc['X_sample'], rtol=0, atol=1e-4)
    mins, _ = dupes.cosine_dedupe_device(X)
    keep = np.nonzero(~(mins <= c['thr']))[0]
    np.testing.assert_array_equal(keep, gc['dedupe_keep'])
    ks = [int(k) for k in gc['k']]
    labels, scores = cluster_sweep(Xh[keep], ks, 0)
    print('c4 chain (%s): N %d, kept %d; rows whose label differs per k %s (sklearn under 1e-5 noise: %s)'
          % (precision, n, len(keep), [int((a != b).sum()) for a, b in zip(labels, gc['labels'])],
             gc['perturbed_rows'].tolist()))
    for i, k in enumerate(ks):
        np.testing.assert_array_equal(labels[i], gc['labels'][i], err_msg='k=%d' % k)
    np.testing.assert_allclose(np.array([s[1:] for s in scores]), gc['scores'], rtol=1e-3)


def test_cosine_dedupe_keep_set_10k():
    """remove_dupes_overall('enc') at N = 10k (configs 4/5 scale): mins, argmins and the keep set
    bit-exact vs the pinned restatement of sklearn's bits (oracle/grouping_oracle.c)."""
    from oracle import grouping as og
    from videotofaces import dupes
    rng = np.random.default_rng(31)
    N, D = 10000, 512
    X = rng.normal(0, 1, (N, D)).astype(np.float32)
    # near-duplicates of earlier rows at cosine distances spread over 0.02 .. 0.5 (both sides of
    # the 0.25 threshold)
    src = rng.integers(0, N // 2, 600)
    dst = rng.choice(np.arange(N // 2, N), 600, replace=False)
    for s_, d_ in zip(src, dst):
        t = rng.uniform(0.02, 0.5)
        noise = rng.normal(0, 1, D).astype(np.float32)
        X[d_] = X[s_] + noise * np.float32(np.sqrt(2 * t / (1 - t)) * 0.999)  # ~ distance t
    mins, inds = dupes.cosine_dedupe_device(torch.from_numpy(X).cuda())
    rm, ri = og.cosine_dedupe(X)
    np.testing.assert_array_equal(mins, rm)
    np.testing.assert_array_equal(inds, ri)
    np.testing.assert_array_equal(mins <= 0.25, rm <= 0.25)
    print('dupes', int((rm <= 0.25).sum()), 'of', N)

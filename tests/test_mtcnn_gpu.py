"""GPU parity: MTCNN on libvtf_hip.so vs the oracle (CPU restatement) and golden vectors made
from the reference modules (tests/golden/make_golden.py)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def g():
    return np.load(os.path.join(GOLDEN, 'mtcnn.npz'))


@pytest.fixture(scope='module')
def model():
    from videotofaces.detectors.mtcnn import MTCNN
    return MTCNN('cuda:0')


@pytest.fixture(scope='module')
def params():
    from videotofaces import synth
    return synth.make_params('mtcnn')


def test_resample_bit_exact_vs_golden(g, model):
    # MTCNN._resample(_preprocess(frame)) -- adaptive_avg_pool2d up- and down-sampling
    fr = torch.from_numpy(g['pyr_frame']).cuda()
    for i, (lh, lw) in enumerate(g['pyr_sizes']):
        out = model.resample(fr, int(lh), int(lw)).cpu().numpy()
        np.testing.assert_array_equal(out, g['pyr_level%d' % i])


def test_pnet_level_vs_oracle(model, params):
    from videotofaces import synth
    from oracle import mtcnn as om
    import torch.nn.functional as F
    fr = synth.make_frames(2, 90, 160, seed=9)
    x = om.preprocess(list(fr))
    dev = torch.from_numpy(fr).cuda()
    for (lh, lw) in [(217, 385), (154, 273), (54, 97), (12, 21), (13, 12)]:
        reg, prob = model.pnet_level(dev, lh, lw)
        rref, pref = om.pnet(params, F.adaptive_avg_pool2d(x, (lh, lw)))
        np.testing.assert_allclose(prob.cpu().numpy(), pref.numpy(), rtol=0, atol=2e-5)
        np.testing.assert_allclose(reg.cpu().numpy(), rref.numpy(), rtol=0, atol=2e-5)


@pytest.mark.parametrize('force_fp32', ['0', '1'])
def test_pnet_paths_vs_oracle(params, force_fp32, monkeypatch):
    # conv2/conv3 of k_pnet run on fp16 matrix cores with split operands by default and on fp32
    # MFMA when VTF_MTCNN_FP32=1 (the fallback for weights whose activations could leave the
    # fp16 range): both within the same fp32-grade tolerance of the oracle
    from videotofaces import synth
    from videotofaces.detectors.mtcnn import MTCNN
    from oracle import mtcnn as om
    import torch.nn.functional as F
    monkeypatch.setenv('VTF_MTCNN_FP32', force_fp32)
    m = MTCNN('cuda:0')
    fr = synth.make_frames(2, 120, 200, seed=21)
    x = om.preprocess(list(fr))
    dev = torch.from_numpy(fr).cuda()
    for (lh, lw) in [(288, 480), (101, 168), (31, 40)]:
        reg, prob = m.pnet_level(dev, lh, lw)
        rref, pref = om.pnet(params, F.adaptive_avg_pool2d(x, (lh, lw)))
        np.testing.assert_allclose(prob.cpu().numpy(), pref.numpy(), rtol=0, atol=2e-5)
        np.testing.assert_allclose(reg.cpu().numpy(), rref.numpy(), rtol=0, atol=2e-5)


@pytest.mark.parametrize('force_fp32', ['0', '1'])
def test_rnet_onet_vs_golden(g, force_fp32, monkeypatch):
    # RNet / ONet convs: split-fp16 conv mode by default, fp32 MFMA with VTF_MTCNN_FP32=1
    from videotofaces.detectors.mtcnn import MTCNN
    monkeypatch.setenv('VTF_MTCNN_FP32', force_fp32)
    model = MTCNN('cuda:0')
    reg, prob = model.rnet(torch.from_numpy(g['rnet_in']))
    np.testing.assert_allclose(reg.cpu().numpy(), g['rnet_reg'], atol=2e-5)
    np.testing.assert_allclose(prob.cpu().numpy(), g['rnet_prob'], atol=2e-5)
    reg, lm, prob = model.onet(torch.from_numpy(g['onet_in']))
    np.testing.assert_allclose(reg.cpu().numpy(), g['onet_reg'], atol=2e-5)
    np.testing.assert_allclose(lm.cpu().numpy(), g['onet_lm'], atol=2e-5)
    np.testing.assert_allclose(prob.cpu().numpy(), g['onet_prob'], atol=2e-5)


def _random_boxes(n, n_img, seed, grid=False):
    rng = np.random.default_rng(seed)
    if grid:  # stage-1-like: integer grid boxes, many exact ties in geometry
        xy = rng.integers(0, 200, (n, 2)).astype(np.float32)
        wh = rng.integers(5, 40, (n, 1)).astype(np.float32)
        b = np.concatenate([xy, xy + wh], 1)
    else:
        xy = rng.uniform(0, 300, (n, 2)).astype(np.float32)
        wh = rng.uniform(2, 80, (n, 2)).astype(np.float32)
        b = np.concatenate([xy, xy + wh], 1)
    s = rng.uniform(0.6, 1.0, n).astype(np.float32)
    s[rng.integers(0, n, n // 10)] = np.float32(0.75)  # ties: stable order matters
    i = rng.integers(0, n_img, n).astype(np.int64)
    return torch.from_numpy(b), torch.from_numpy(s), torch.from_numpy(i)


@pytest.mark.parametrize('n,n_img,thr,grid', [(0, 1, 0.5, False), (1, 1, 0.5, False), (300, 4, 0.5, True),
                                              (1000, 3, 0.7, False), (1001, 3, 0.7, False), (5000, 16, 0.5, True),
                                              (3000, 1, 0.45, False), (20000, 7, 0.3, True), (16384, 1, 0.7, False),
                                              (9000, 2, 0.6, True), (66000, 8, 0.5, False)])
def test_batched_nms_exact(n, n_img, thr, grid):
    """Calls of up to 65536 boxes take the per-segment sort (segments of up to 4096 boxes in LDS,
    longer ones -- 16384 in one image -- in global memory); larger calls (66000) the device-wide
    merge sort; all give the same order."""
    from videotofaces.detectors.mtcnn import batched_nms
    from oracle import nms as onms
    b, s, i = _random_boxes(n, n_img, seed=n + n_img, grid=grid)
    ref = onms.batched_nms(b, s, i, thr)
    got = batched_nms(b.cuda(), s.cuda(), i.cuda(), thr).cpu()
    # exact order on both paths: above 1000 boxes (vanilla) the reference's final order is
    # torch's unstable CPU sort, whose order among the tied scores (10 % of the boxes share 0.75)
    # the library reproduces (nms.hpp torch_unstable_desc_order)
    assert got.tolist() == ref.tolist()
    if n > 1000:
        ks = s[ref]
        print('vanilla path: %d kept, %d equal-score neighbours' % (len(ref), int((ks[1:] == ks[:-1]).sum())))


def test_batched_nms_degenerate_boxes_exact():
    """Zero-area, inverted (x2 < x1) and NaN boxes: their unions are <= 0 or NaN, so k_iou_mask
    decides those pairs by the reference's IEEE division instead of the division-free test."""
    from videotofaces.detectors.mtcnn import batched_nms
    from oracle import nms as onms
    b, s, i = _random_boxes(3000, 3, seed=5, grid=True)
    b = b.clone()
    b[::7, 2] = b[::7, 0]                    # zero width
    b[1::11, 2] = b[1::11, 0] - 3.0          # inverted
    b[2::13, 3] = b[2::13, 1] - 1.0
    b[3::97, 0] = float('nan')               # NaN coordinate
    for n in (3000, 900):                    # vanilla and coordinate-trick paths
        ref = onms.batched_nms(b[:n], s[:n], i[:n], 0.5)
        got = batched_nms(b[:n].cuda(), s[:n].cuda(), i[:n].cuda(), 0.5).cpu()
        assert got.tolist() == ref.tolist()


@pytest.mark.parametrize('n', [3000, 900])
def test_batched_nms_nan_scores_exact(n):
    """NaN scores sort above every number and tie among themselves (torch's sort); on the vanilla
    path the kept NaNs are ties the host reorders like torch's unstable final sort."""
    from videotofaces.detectors.mtcnn import batched_nms
    from oracle import nms as onms
    b, s, i = _random_boxes(n, 3, seed=11, grid=False)
    s = s.clone()
    s[::37] = float('nan')
    s[5::41] = -float('nan')
    ref = onms.batched_nms(b, s, i, 0.5)
    got = batched_nms(b.cuda(), s.cuda(), i.cuda(), 0.5).cpu()
    assert got.tolist() == ref.tolist()


@pytest.mark.parametrize('n,base,spread', [(3000, 20000, 7), (900, 20000, 3), (17000, 5, 17000)])
def test_batched_nms_large_and_many_class_ids(n, base, spread):
    """Category ids far above the box count (torchvision takes any id): the vanilla path (n > 1000)
    groups by id only, so the library remaps the ids to dense ranks; the coordinate-trick path
    (900 boxes) keeps the values, which set its offsets' fp32 rounding.  17,000 distinct ids give
    more segments than k_nms_out's LDS prefix holds (15,000): the prefix comes from global memory
    and the call takes the merge sort."""
    from videotofaces.detectors.mtcnn import batched_nms
    from oracle import nms as onms
    b, s, _ = _random_boxes(n, 1, seed=n + spread, grid=True)
    rng = np.random.default_rng(n)
    ids = rng.permutation(n) if spread >= n else rng.integers(0, spread, n)  # (all distinct: S = n)
    i = torch.from_numpy((base + ids).astype(np.int64))
    ref = onms.batched_nms(b, s, i, 0.5)
    got = batched_nms(b.cuda(), s.cuda(), i.cuda(), 0.5).cpu()
    assert got.tolist() == ref.tolist()


@pytest.mark.parametrize('n', [3000, 900])
def test_batched_nms_signed_zero_scores_exact(n):
    """-0 and +0 scores compare equal in torch's sort: a stable order keeps them by index and the
    vanilla path's final unstable sort treats them as a tie (desc_key maps -0 to +0's key)."""
    from videotofaces.detectors.mtcnn import batched_nms
    from oracle import nms as onms
    b, s, i = _random_boxes(n, 3, seed=17, grid=True)
    s = s.clone()
    s[::5] = -0.0
    s[1::5] = 0.0
    ref = onms.batched_nms(b, s, i, 0.5)
    got = batched_nms(b.cuda(), s.cuda(), i.cuda(), 0.5).cpu()
    assert got.tolist() == ref.tolist()


def _match(res, counts, boxes, atol):
    k = 0
    for r, c in zip(res, counts):
        assert r.shape == (c, 5), (r.shape, c)
        np.testing.assert_allclose(r, boxes[k:k + c], atol=atol, rtol=1e-5)
        k += c


def test_detect_small_frames_vs_golden(g, model):
    res = model(list(g['small_frames']), 5)
    _match(res, g['small_ms5_counts'], g['small_ms5_boxes'], 2e-3)


@pytest.mark.parametrize('ms', [5, 20])
def test_detect_720p_vs_golden(g, model, ms):
    from videotofaces import synth
    frames = synth.make_frames(2, seed=int(g['e2e_frames_seed'][0]))
    res, ldm = model(frames, ms, return_landmarks=True)
    _match(res, g['e2e_ms%d_counts' % ms], g['e2e_ms%d_boxes' % ms], 2e-3)
    np.testing.assert_allclose(np.concatenate(ldm), g['e2e_ms%d_landmarks' % ms], atol=2e-3, rtol=1e-5)


def test_detect_device_frames_and_strided_view(model):
    # borrowed non-contiguous view (video_area slice, detection.py:114-116) and HBM frames
    from videotofaces import synth
    fr = synth.make_frames(2, 200, 300, seed=4)
    view = fr[:, 10:190, 20:280, :]
    a = model(view, 5)
    b = model(np.ascontiguousarray(view), 5)
    c = model(torch.from_numpy(np.ascontiguousarray(view)).cuda(), 5)
    for x, y, z in zip(a, b, c):
        np.testing.assert_array_equal(x, y)
        np.testing.assert_array_equal(x, z)


@pytest.mark.parametrize('case', ['crafted', 'dense', 'sparse'])
def test_iom_chain_nms_vs_reference(case):
    """A-M12 edge cases: MTCNN._nms_vectorized(..., 0.7, 'Min') of the reference (chains, one-pixel
    touches counted by the +1 widths, IoM exactly 0.7 kept, identical and nested boxes, several
    classes) -- the device kernel (vtf_iom_nms) keeps exactly the same rows in the same order."""
    from videotofaces.detectors.mtcnn import nms_iom
    gi = np.load(os.path.join(GOLDEN, 'iom.npz'))
    b, s, c = (torch.from_numpy(gi[case + k]).cuda() for k in ('_boxes', '_scores', '_classes'))
    keep = nms_iom(b, s, c, 0.7).cpu().numpy()
    np.testing.assert_array_equal(keep, gi[case + '_keep'])


@pytest.mark.parametrize('ms', [5, 20])
def test_fused_candidate_nets_match_layer_path(ms, monkeypatch):
    """The fused RNet/ONet front half (crop .. conv2 + pool2 in LDS, mtcnn_cand.hip; opt-in with
    VTF_MTCNN_FUSED=1) against the default layer-by-layer path on the same 720p frames: same
    detections, boxes and scores within the fp32-grade tolerance of the e2e golden test."""
    from videotofaces import synth
    from videotofaces.detectors.mtcnn import MTCNN
    fr = torch.from_numpy(synth.make_frames(4, seed=21)).cuda()
    b = MTCNN('cuda:0')(fr, ms)
    monkeypatch.setenv('VTF_MTCNN_FUSED', '1')
    a = MTCNN('cuda:0')(fr, ms)
    assert [x.shape for x in a] == [y.shape for y in b]
    for x, y in zip(a, b):
        np.testing.assert_allclose(x, y, rtol=1e-5, atol=2e-3)


@pytest.mark.parametrize('ms', [5, 20])
def test_span_convs_match_gather_path(ms, monkeypatch):
    """RNet conv2 / ONet conv2 / conv3 on the span kernel (k_conv_span: the tile's contiguous input
    run staged once, conv_dma.hip; default) against the implicit-GEMM gather (VTF_CONV_SPAN=0) on
    the same 720p frames: same detections, boxes and scores within the fp32-grade tolerance of the
    e2e golden test (same k order and MFMA chains; the gather path's tail tiles split K)."""
    from videotofaces import synth
    from videotofaces.detectors.mtcnn import MTCNN
    fr = torch.from_numpy(synth.make_frames(4, seed=23)).cuda()
    m = MTCNN('cuda:0')
    a = m(fr, ms)
    monkeypatch.setenv('VTF_CONV_SPAN', '0')
    b = m(fr, ms)
    assert [x.shape for x in a] == [y.shape for y in b]
    assert sum(x.shape[0] for x in a) > 0
    for x, y in zip(a, b):
        np.testing.assert_allclose(x, y, rtol=1e-5, atol=2e-3)


@pytest.mark.parametrize('ms', [5, 20])
def test_span_pool_fusion_matches_separate_pool(ms, monkeypatch):
    """RNet conv2 + pool1 and ONet conv2 + pool1 as one launch (k_conv_span_pool: pool-aligned
    tiles, the conv map kept in LDS, only the pooled split pairs written; default) against the
    span conv + separate max-pool launch (VTF_CONV_SPAN_POOL=0): same detections, boxes and scores
    within the e2e tolerance (the same conv sums; the pool and the split are exact)."""
    from videotofaces import synth
    from videotofaces.detectors.mtcnn import MTCNN
    fr = torch.from_numpy(synth.make_frames(4, seed=29)).cuda()
    m = MTCNN('cuda:0')
    a = m(fr, ms)
    monkeypatch.setenv('VTF_CONV_SPAN_POOL', '0')
    b = m(fr, ms)
    assert [x.shape for x in a] == [y.shape for y in b]
    assert sum(x.shape[0] for x in a) > 0
    for x, y in zip(a, b):
        np.testing.assert_allclose(x, y, rtol=1e-5, atol=2e-3)


@pytest.mark.parametrize('ms', [5, 20])
def test_wave_front_bit_identical(ms, monkeypatch):
    """The RNet candidate front as one wave per candidate (k_cand_front_w24, default) against one
    workgroup per candidate (VTF_FRONT_WAVE=0): the same crop bins, conv1 MFMA chains, PReLU, pool
    and split, so the detections are identical bit for bit."""
    from videotofaces import synth
    from videotofaces.detectors.mtcnn import MTCNN
    fr = torch.from_numpy(synth.make_frames(4, seed=31)).cuda()
    m = MTCNN('cuda:0')
    a = m(fr, ms)
    monkeypatch.setenv('VTF_FRONT_WAVE', '0')
    b = m(fr, ms)
    assert sum(x.shape[0] for x in a) > 0
    for x, y in zip(a, b):
        np.testing.assert_array_equal(x, y)

"""GPU parity: Faster R-CNN anime-face detector on libvtf_hip.so vs reference goldens / oracle.

Tolerances (north_star: fp32 within 1e-4): the preprocess is bit-exact against the
restatement; RPN head maps of a small input within 1e-4 x max|map| (53 + 11 fp32 convs, MFMA
summation order vs oneDNN's); roi_align bit-exact against the torchvision restatement on the
same maps; end to end from frames, the same proposal set up to a few boundary swaps of the
per-level top-1000 (logits within 1e-5 of each other), the same detection counts, boxes
within 1e-2 px and scores within 1e-4.
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def g():
    return np.load(os.path.join(GOLDEN, 'rcnn.npz'))


@pytest.fixture(scope='module')
def det():
    from videotofaces.detectors.rcnn import FasterRCNN
    return FasterRCNN('cuda:0', precision='fp32')


@pytest.mark.parametrize('hw', [(720, 1280), (1080, 1920), (180, 320), (750, 1333)])
def test_preprocess_bit_exact(det, hw):
    from videotofaces import synth
    from oracle import rcnn as orc
    fr = synth.make_frames(2, hw[0], hw[1], seed=4)
    out = det.preprocess(torch.from_numpy(fr).cuda()).cpu()
    x, so, su = orc.preprocess(list(fr))
    assert out.shape[1:3] == x.shape[2:]
    np.testing.assert_array_equal(out[..., :3].permute(0, 3, 1, 2).numpy(), x.numpy())
    assert not out[..., 3:].any()


def test_rpn_heads_small_vs_golden(det, g):
    heads = det.rpn_heads(torch.from_numpy(g['small_x']))
    for i, (reg, log) in enumerate(heads):
        for name, t in (('reg', reg), ('log', log)):
            ref = g['small_%s%d' % (name, i)]
            err = np.abs(t.cpu().numpy() - ref).max()
            print('level %d %s max err %.3g (scale %.3g)' % (i, name, err, np.abs(ref).max()))
            np.testing.assert_allclose(t.cpu().numpy(), ref, rtol=0, atol=1e-4 * np.abs(ref).max())


def test_roi_align_bit_exact(g):
    from videotofaces.detectors.rcnn import roi_align
    out = roi_align(torch.from_numpy(g['ra_fmap']).cuda(), torch.from_numpy(g['ra_rois']).cuda(), 0.25)
    np.testing.assert_array_equal(out.cpu().numpy(), g['ra_out'])


def test_roi_align_random_vs_oracle():
    from oracle import rcnn as orc
    from videotofaces.detectors.rcnn import roi_align
    gen = torch.Generator().manual_seed(3)
    fmap = torch.randn(3, 32, 48, 84, generator=gen)
    xy = torch.rand(40, 2, generator=gen) * torch.tensor([1344.0, 768.0])
    wh = torch.rand(40, 2, generator=gen) * 400
    rois = torch.cat([torch.randint(0, 3, (40, 1), generator=gen).float(), xy, xy + wh], 1)
    out = roi_align(fmap.cuda(), rois.cuda(), 1 / 16).cpu()
    np.testing.assert_array_equal(out.numpy(), orc.roi_align(fmap, rois, 7, 1 / 16, True).numpy())


def _match_rows(a, b, atol):
    """fraction of rows of a with a row of b within atol (order-free)."""
    if len(a) == 0:
        return 1.0
    d = np.abs(a[:, None, :] - b[None, :, :]).max(-1)
    return float((d.min(1) <= atol).mean())


def test_rpn_selection_exact_on_same_heads(det):
    """A-R2's integer path on identical inputs: the device RPN selection (per-level top-1000,
    decode, clamp, remove_small, batched_nms(0.7) by (image, level), top-1000 per image;
    rcnn.py:49-82) and the oracle's restatement (pinned to the reference's own RPN by
    tests/golden/rcnn.npz) fed the SAME head maps of two 720p frames keep the same proposals in
    the same order (boxes within 1e-3 px: exp() ulps in the decode).  The order is decided by
    the objectness sigmoid(logit) in fp32 (batched_nms's stable score sort); both sides compute
    torch's CPU sigmoid bit for bit (Sleef expf on vector steps, glibc expf on the chunk tail:
    rcnn.hip torch_sigmoid, oracle.rcnn.torch_sigmoid_survey), so no proposal moves."""
    from videotofaces import synth
    from videotofaces.detectors.rcnn import input_size
    from oracle import rcnn as orc
    fr = torch.from_numpy(synth.make_frames(2, seed=0)).cuda()
    hu, wu, Hp, Wp = input_size(720, 1280)
    x = det.preprocess(fr)[..., :3].permute(0, 3, 1, 2).contiguous()
    heads = det.rpn_heads(x, raw=True)
    pb, pi = det.rpn_proposals(heads, Hp, Wp, hu, wu)
    regs, logs = [], []
    for t in heads:
        t = t.cpu().reshape(2, -1, 15)
        logs.append(t[..., :3].reshape(2, -1, 1))
        regs.append(t[..., 3:].reshape(2, -1, 4))
    with torch.inference_mode():
        rb, ri = orc.rpn_select(regs, logs, orc.priors((Hp, Wp)), [(hu, wu)] * 2)
    rb, ri = rb.numpy(), ri.numpy()
    np.testing.assert_array_equal(pi, ri)
    moved = 0
    for i in range(2):
        a, b = pb[pi == i], rb[ri == i]
        oa, ob = np.lexsort(a.T[::-1]), np.lexsort(b.T[::-1])
        np.testing.assert_allclose(a[oa], b[ob], rtol=0, atol=1e-3)
        moved += int((np.abs(a - b).max(1) > 1e-3).sum())
    print('proposals', len(pb), 'at a different position', moved)
    assert moved == 0


def test_detect_e2e_vs_golden(det, g):
    from videotofaces import synth
    fr = synth.make_frames(2, seed=0)
    b, s, c = det(fr)
    props, pimg = det.proposals()
    # RPN from frames: same per-image proposal counts and the same proposal set (order-free, boxes
    # within 1e-2 px).  The head convs' fp32 summation order differs from oneDNN's, so in general
    # two logits closer than that noise at a per-level top-1000 boundary (193,536 anchors at level
    # 0) could trade places; on this fixture none do, and the selection itself is exact on
    # identical heads (test_rpn_selection_exact_on_same_heads)
    for i in range(2):
        pa, pb = props[pimg == i], g['proposals'][g['prop_imidx'] == i]
        assert len(pa) == len(pb)
        frac = _match_rows(pa, pb, 1e-2)
        print('image %d proposals matched %.4f' % (i, frac))
        assert frac == 1.0
    assert [len(t) for t in s] == list(g['counts'])
    np.testing.assert_allclose(np.concatenate(b), g['boxes'], rtol=1e-6, atol=1e-2)
    np.testing.assert_allclose(np.concatenate(s), g['scores'], rtol=1e-6, atol=1e-4)
    np.testing.assert_array_equal(np.concatenate(c), g['classes'])
    # frames already in HBM, as a strided view: identical results
    big = torch.zeros((2, 720, 1400, 3), dtype=torch.uint8)
    big[:, :, 60:1340] = torch.from_numpy(fr)
    b2, s2, _ = det(big.cuda()[:, :, 60:1340])
    for x, y in zip(b, b2):
        np.testing.assert_array_equal(x, y)


def test_detect_small_frames_vs_oracle(det):
    """a different frame size and batch of 3 against the oracle end to end."""
    from videotofaces import synth
    from oracle import rcnn as orc
    fr = synth.make_frames(3, 180, 320, seed=9)
    b, s, _ = det(fr)
    rb, rs, _ = orc.forward(synth.make_params('rcnn'), list(fr))
    assert [len(t) for t in s] == [len(t) for t in rs]
    for x, y, xs, ys in zip(b, rb, s, rs):
        if len(y):
            np.testing.assert_allclose(x, y, rtol=1e-5, atol=1e-2)
            np.testing.assert_allclose(xs, ys, rtol=1e-4, atol=1e-6)


def test_bf16_detect_runs(g):
    from videotofaces.detectors.rcnn import FasterRCNN
    from videotofaces import synth
    m = FasterRCNN('cuda:0', precision='bf16')
    heads = m.rpn_heads(torch.from_numpy(g['small_x']))
    for i, (reg, log) in enumerate(heads):
        ref = g['small_log%d' % i]
        rel = np.abs(log.cpu().numpy() - ref).max() / np.abs(ref).max()
        print('bf16 level %d logit rel err %.3g' % (i, rel))
        assert rel < 0.1
    b, s, _ = m(synth.make_frames(2, seed=0))
    print('bf16 counts', [len(t) for t in s], 'fp32 golden', list(g['counts']))

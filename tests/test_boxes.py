"""Box post-processing between detector and encoder (detection.py:126-262).

CPU: the oracle's vectorised restatement (oracle/boxes.py) against the reference's own
filter_boxes / adjust_boxes on 10,500 random and edge-case boxes (tests/golden/boxes.npz).
GPU: the device kernel (vtf_boxes_to_crops, csrc/boxes.hip) against the same fixture, bit-exact,
with the rows split over several frames (order, frame offsets, empty and absent frames), and the
detectors' device crop path (vtf_*_detect_crops) against host detection + the kernel."""
import json
import os

import numpy as np
import pytest

from conftest import GOLDEN


@pytest.fixture(scope='module')
def g():
    return np.load(os.path.join(GOLDEN, 'boxes.npz'))


def _cases(g):
    return [tuple(c) for c in json.loads(str(g['cases_json']))]


def test_oracle_boxes_vs_reference(g):
    from oracle import boxes as ob
    for ci, (sz, ms, mz, mb, sc, sq) in enumerate(_cases(g)):
        rows = g['rows%d' % ci]
        sc = sc if isinstance(sc, int) else tuple(sc)
        keep = ob.passes(rows, sz, ms, mz, mb)
        x1, y1, x2, y2, s = ob._round_out(rows[keep])
        np.testing.assert_array_equal(np.stack([x1, y1, x2, y2], 1), g['filtered%d' % ci], err_msg='case %d' % ci)
        np.testing.assert_array_equal(s, g['filtered_score%d' % ci])
        adj = np.stack(ob.adjust(x1, y1, x2, y2, sz, sc, sq), 1)
        np.testing.assert_array_equal(adj, g['adjusted%d' % ci], err_msg='case %d' % ci)
        crops, src = ob.rows_to_crops([rows], sz, ms, mz, mb, sc, sq, frame_offset=3)
        np.testing.assert_array_equal(crops[:, 1:], g['adjusted%d' % ci])
        assert np.all(crops[:, 0] == 3)


def _split(rows, rng, B):
    """rows -> B frames (some empty) with the same concatenated order"""
    cuts = np.sort(rng.integers(0, rows.shape[0] + 1, B - 1))
    return np.split(rows, cuts)


@pytest.mark.gpu
def test_box_kernel_vs_reference(g):
    from videotofaces import _native as nat
    from videotofaces.detection import _rows_to_crops
    from oracle import boxes as ob
    rng = np.random.default_rng(5)
    for ci, (sz, ms, mz, mb, sc, sq) in enumerate(_cases(g)):
        rows = g['rows%d' % ci]
        sc = sc if isinstance(sc, int) else tuple(sc)
        # one frame: exact vs the reference fixture, filter-only and the full pipeline
        cr, src, fc = _rows_to_crops([rows], sz, nat.BoxParams.make(ms, mz, mb, adjust=False))
        np.testing.assert_array_equal(cr[:, 1:], g['filtered%d' % ci], err_msg='filter case %d' % ci)
        np.testing.assert_array_equal(rows[src, 4], g['filtered_score%d' % ci])
        cr, src, fc = _rows_to_crops([rows], sz, nat.BoxParams.make(ms, mz, mb, sc, sq), frame_offset=7)
        np.testing.assert_array_equal(cr[:, 1:], g['adjusted%d' % ci], err_msg='adjust case %d' % ci)
        assert np.all(cr[:, 0] == 7) and fc.tolist() == [cr.shape[0]]
        # many frames (incl. empty ones): (frame, face) order and per-frame counts vs the oracle
        for B in (2, 17, 300):
            parts = _split(rows, rng, B)
            cr, src, fc = _rows_to_crops(parts, sz, nat.BoxParams.make(ms, mz, mb, sc, sq), frame_offset=11)
            ref, _ = ob.rows_to_crops(parts, sz, ms, mz, mb, sc, sq, frame_offset=11)
            np.testing.assert_array_equal(cr, ref, err_msg='case %d B %d' % (ci, B))
            np.testing.assert_array_equal(fc, np.bincount(ref[:, 0] - 11, minlength=B))


@pytest.mark.gpu
def test_box_kernel_api_wrappers(g):
    """detection.filter_boxes / adjust_boxes (reference signatures) run on the kernel."""
    from videotofaces import detection
    sz, ms, mz, mb, sc, sq = _cases(g)[0]
    rows = g['rows0']
    kept = detection.filter_boxes(rows, sz, ms, mz, mb, ('', '', None, False, False, False), None, 0)
    np.testing.assert_array_equal(np.array([b[:4] for b in kept]), g['filtered0'])
    adj = detection.adjust_boxes(kept, sz, tuple(sc), sq)
    np.testing.assert_array_equal(np.array([b[:4] for b in adj]), g['adjusted0'])
    assert [b[4] for b in adj] == [b[4] for b in kept]
    assert detection.boxes_to_crops([rows[:0]], sz).shape == (0, 5)


@pytest.mark.gpu
@pytest.mark.parametrize('det', ['mtcnn', 'yolo', 'rcnn'])
def test_detect_crops_matches_host_path(det):
    """vtf_*_detect_crops (detector rows never leave HBM) == host detection + box kernel."""
    import torch
    from videotofaces import synth
    from videotofaces.detection import boxes_to_crops, detect_crops, normalize_detout
    frames = synth.make_frames(3, 360, 640, seed=9)
    fr = torch.from_numpy(frames).cuda()
    if det == 'mtcnn':
        from videotofaces.detectors.mtcnn import RealMTCNN
        m = RealMTCNN('cuda:0', min_face_size=10)
    elif det == 'yolo':
        from videotofaces.detectors.yolo import RealYOLO
        m = RealYOLO('cuda:0')
    else:
        from videotofaces.detectors.rcnn import AnimeFRCNN
        m = AnimeFRCNN('cuda:0')
    params = dict(mscore=0.2, msize=0, mborder=2, scale=(1.5, 1.5, 2.2, 1.2), square=True)
    host = boxes_to_crops(normalize_detout(m(fr)), (360, 640), frame_offset=4, **params)
    d, counts = detect_crops(m, fr, 4, **params)
    np.testing.assert_array_equal(d.cpu().numpy(), host)
    np.testing.assert_array_equal(counts, np.bincount(host[:, 0] - 4, minlength=3) if len(host) else np.zeros(3))

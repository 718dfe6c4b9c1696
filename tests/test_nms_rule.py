"""CPU: the division-free IoU decision of k_iou_mask (csrc/nms.hip) -- inter > mid * uni (or >=
when F's significand is even) in double -- equals the reference's (double)fl(inter / uni) > thr
(torchvision nms_kernel.cpp: float IoU promoted to double) on random and on constructed
near-threshold float pairs, for the thresholds the reference uses (mtcnn.py:196,205,219;
post.py:8) and a few others."""
import numpy as np
import pytest


def iou_thr(thr):
    f = np.float32(thr)
    if not float(f) > thr:
        f = np.nextafter(f, np.float32(np.inf))
    fm = np.nextafter(f, np.float32(-np.inf))
    ge = (int(np.array(f, np.float32).view(np.uint32)) & 1) == 0
    return (float(fm) + float(f)) * 0.5, ge, f, fm


@pytest.mark.parametrize('thr', [0.5, 0.7, 0.45, 0.3, 0.6, 1.0 / 3.0, 0.0])
def test_division_free_rule_matches_division(thr):
    mid, ge, f, fm = iou_thr(thr)
    rng = np.random.default_rng(int(thr * 1000))
    uni = (rng.random(200000) * 10.0 ** rng.integers(-3, 7, 200000)).astype(np.float32) + np.float32(1e-6)
    # random ratios around thr, plus pairs at the rounding boundary: inter = round(mid * uni) and
    # its float neighbours
    q = np.concatenate([rng.random(100000), thr + (rng.random(100000) - 0.5) * 1e-6]).astype(np.float64)
    inter = (q * uni.astype(np.float64)).astype(np.float32)
    edge = (mid * uni.astype(np.float64)).astype(np.float32)
    inter = np.concatenate([inter, edge, np.nextafter(edge, np.float32(np.inf)), np.nextafter(edge, np.float32(0))])
    u = np.concatenate([uni, uni, uni, uni])
    ref = (inter / u).astype(np.float32).astype(np.float64) > thr
    l, r = inter.astype(np.float64), mid * u.astype(np.float64)
    got = l >= r if ge else l > r
    assert np.array_equal(got, ref), int((got != ref).sum())
    assert ref.any() and not ref.all()

"""k_pnet's div_small (csrc/mtcnn_kernels.hip) replaces the adaptive-pool bin divisions of the
downsampled levels by an fma-corrected reciprocal:  q = RN(x y), r = RN(fma(-q, k, x)),
q1 = RN(fma(r, y, q)) with y = RN(1/k).  The level pixels must equal the reference's
adaptive_avg_pool2d bits (the pyramid levels are F.adaptive_avg_pool2d of the frame,
/root/reference/src/videotofaces/detectors/mtcnn.py:151), so the quotient must be
the correctly rounded fp32 division for every input the kernel can see: bin sums x = s 2^-8 of
8-bit pixels, |s| <= 2295 (at most 3 x 3 pixels of 255), bin extents k = 1..3, and the row
average divided again by the column extent.  Exhaustive over that domain in exact rational
arithmetic (no GPU)."""
from fractions import Fraction as F

import numpy as np


def _rn32(v):
    """Exact rational -> nearest float32, ties to even (guards against double rounding)."""
    if v == 0:
        return 0.0
    c = np.float32(float(v))
    cands = [np.nextafter(c, np.float32(-np.inf)), c, np.nextafter(c, np.float32(np.inf))]
    best = min(cands, key=lambda t: (abs(F(float(t)) - v),
                                      int(np.frombuffer(np.float32(t).tobytes(), np.uint32)[0]) & 1))
    return float(best)


_Y = {k: _rn32(F(1, k)) for k in (1, 2, 3)}


def _div_small(x, k):
    y = _Y[k]
    q = _rn32(F(x) * F(y))
    r = _rn32(-F(q) * k + F(x))
    return _rn32(F(r) * F(y) + F(q))


def test_div_small_is_correctly_rounded_on_the_bin_domain():
    bad, n = [], 0
    for s in range(-2295, 2296):
        x = float(np.float32(s) * np.float32(2.0 ** -8))
        for kh in (1, 2, 3):
            e = _rn32(F(x) / kh)
            n += 1
            if _div_small(x, kh) != e:
                bad.append((s, kh))
            for kw in (1, 2, 3):
                n += 1
                if _div_small(e, kw) != _rn32(F(e) / kw):
                    bad.append((s, kh, kw))
    assert n == 55092
    assert not bad, bad[:10]


def test_plain_reciprocal_product_is_not_enough():
    """The correction step is needed: RN(x * RN(1/3)) differs from RN(x / 3) somewhere."""
    diffs = sum(_rn32(F(float(np.float32(s) * np.float32(2.0 ** -8))) * F(_Y[3]))
                != _rn32(F(float(np.float32(s) * np.float32(2.0 ** -8))) / 3)
                for s in range(1, 2296))
    assert diffs > 0

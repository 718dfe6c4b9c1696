"""Exhaustive check of k_pnet div_small (mtcnn_kernels.hip): the fma-corrected reciprocal quotient
equals the correctly rounded fp32 division for every adaptive-pool bin average of the downsampled
levels (x = s 2^-8, |s| <= 2295, k in 1..3) and for every such quotient divided again.  Exact rational
arithmetic (fractions); prints the mismatch count (0)."""
# exhaustive check: fast exact division of the adaptive-pool bin averages
# q = RN(x*y); r = RN(fma(-q, k, x)) ; q1 = RN(fma(r, y, q))  vs RN(x/k), y = RN(1/k), float32, RNE
from fractions import Fraction as F
import numpy as np, struct
def rn32(v):  # exact rational -> nearest float32 (ties to even)
    if v == 0: return 0.0
    f = float(v)  # nearest double (exact rational rounding by Python)
    c = np.float32(f)
    # correct double rounding: compare candidates around c
    cands = [np.nextafter(c, np.float32(-np.inf)), c, np.nextafter(c, np.float32(np.inf))]
    best = min(cands, key=lambda t: (abs(F(float(t)) - v), int(np.frombuffer(np.float32(t).tobytes(), np.uint32)[0]) & 1))
    return float(best)
bad = 0; n = 0
ys = {k: rn32(F(1, k)) for k in (1, 2, 3)}
def fdiv(x, k):
    y = ys[k]
    q = rn32(F(x) * F(y))
    r = rn32(-F(q) * k + F(x))
    return rn32(F(r) * F(y) + F(q))
for s in range(-2295, 2296):
    x = float(np.float32(s) * np.float32(0.00390625))
    for kh in (1, 2, 3):
        a = fdiv(x, kh); e = rn32(F(x) / kh); n += 1
        if a != e: bad += 1
        for kw in (1, 2, 3):
            b = fdiv(e, kw); e2 = rn32(F(e) / kw); n += 1
            if b != e2: bad += 1
print('cases', n, 'mismatches', bad)

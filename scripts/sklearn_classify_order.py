"""Measure the float32 orders behind classify's cosine_distances(X, R) (grouping.py:51) in this
container: X_n @ R_n.T is numpy matmul on two buffers -> numpy's OpenBLAS 0.3.29 (SkylakeX):
  * sgemm (both sides > 1 row): the E-step's rules (sklearn_order.py) -- checked by the oracle test;
  * sgemv_t (one side a single row) and sdot (both single rows): probed here.
1. Absorption: 2^30 at position i, -2^30 at j, 1 at t: the result is 1 iff i and j cancel before
   t joins either -> lanes and the lane tree.
2. Kernel per output: an 8-vs-4-lane probe (2^30 at 0, -2^30 at 8, 1 at 4) and an fma probe
   ((-1) + (1 + 2^-15)^2: fma keeps 2^-14 + 2^-30, product-then-add gives 2^-14) classify every
   output as the 4x4 (8 lanes, fma), 4x2 (4 lanes, mul + add) or 4x1 (8 lanes, mul + add) kernel;
   runs of them reveal OpenBLAS's thread split of the outputs (D n >= 460800: 8 threads here).
Restated in oracle/grouping_oracle.c (ora_cos_classify_dist) and csrc/grouping.hip (k_classify).

    python scripts/sklearn_classify_order.py
"""
import numpy as np

B = np.float32(2.0 ** 30)


def ranges(ts):
    out = []
    for t in ts:
        if out and t == out[-1][1] + 1:
            out[-1][1] = t
        else:
            out.append([t, t])
    return out


def probe(D, i, j, m, row, vecmat=False):
    ones = []
    for t in range(D):
        if t in (i, j):
            continue
        A = np.zeros((m, D), np.float32)
        for p, v in ((i, B), (j, -B), (t, 1)):
            A[row, p] = v
        ones_v = np.ones((1, D), np.float32)
        g = (ones_v @ A.T)[0, row] if vecmat else (A @ ones_v.T)[row, 0]
        if g == 1:
            ones.append(t)
    return ranges(ones)


def kinds(N, D):
    X = np.zeros((N, D), np.float32)
    R = np.ones((1, D), np.float32)
    X[:, 0], X[:, 8], X[:, 4] = B, -B, 1
    g1 = (X @ R.T)[:, 0]
    e = np.float32(1 + 2.0 ** -15)
    X = np.zeros((N, D), np.float32)
    X[:, 0], X[:, 8] = -1, e
    R = np.ones((1, D), np.float32)
    R[0, 8] = e
    g2 = (X @ R.T)[:, 0]
    k = np.where(g1 != 1, '2', np.where(g2 == np.float32(2.0 ** -14), '1', '4'))
    runs = []
    for ch in k:
        if runs and runs[-1][0] == ch:
            runs[-1][1] += 1
        else:
            runs.append([ch, 1])
    return ' '.join('4x%s*%d' % (c, n) for c, n in runs)


def main():
    D = 512
    print('sgemv 4x4 kernel (row 0 of 5 x D @ D x 1):')
    for ij in [(0, 1), (0, 2), (0, 4), (0, 8), (0, 16)]:
        print('  ', ij, probe(D, *ij, m=5, row=0)[:6])
    print('sgemv 4x1 kernel (row 4):', [probe(D, 0, j, m=5, row=4)[:3] for j in (1, 8)])
    print('sgemv 4x2 kernel (row 0 of 3 x D):', [probe(D, 0, j, m=3, row=0)[:3] for j in (1, 4, 8)])
    print('sdot (1 x D @ D x 1):')
    for ij in [(0, 1), (0, 8), (0, 16), (0, 32), (0, 48), (0, 64), (16, 32)]:
        print('  ', ij, probe(D, *ij, m=1, row=0)[:8])
    print('kernel per output (4x4 / 4x2 / 4x1 runs):')
    for N in (7, 150, 899, 900, 1000, 1003, 2500):
        print('   N %5d D %d: %s' % (N, D, kinds(N, D)[:160]))


if __name__ == '__main__':
    main()

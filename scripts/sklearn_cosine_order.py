"""Measure the float32 order behind sklearn's cosine_distances(X) (the embedding dedupe of
remove_dupes_overall, dupes.py:60-62) in this container, and check the C restatement
(oracle/grouping_oracle.c) that the device kernels (csrc/grouping.hip) follow.

cosine_similarity normalises X (row_norms = np.einsum, see sklearn_order.py) and computes
X_n @ X_n.T; numpy's matmul sees one buffer times its transpose and calls cblas_ssyrk.

1. Absorption probes on the Gram entry (r, c): x_r holds 2^30 at i, -2^30 at j and 1 at t,
   x_c holds 1 at i, j, t; the entry is 1 iff i and j cancel before t joins them.  Adjacent
   (i, j) = (b-1, b) that do NOT cancel mark a K-block boundary at b.
2. The restatement is then compared with sklearn on every entry of random matrices.

    python scripts/sklearn_cosine_order.py
"""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'video-to-faces_amd')]
from oracle import grouping as og  # noqa: E402

B = np.float32(2.0 ** 30)


def entry(N, D, r, c, i, j, t):
    X = np.zeros((N, D), np.float32)
    X[r, i], X[r, j], X[r, t] = B, -B, 1
    X[c, i] = X[c, j] = X[c, t] = 1
    return round(float((X @ X.T)[r, c]))


def block_bounds(N, D, r=3, c=1):
    return [b for b in range(1, D - 1) if entry(N, D, r, c, b - 1, b, b + 1) != 1]


def sequential(N, D, i, j, r=3, c=1):
    """t positions (outside i, j) that join after i and j cancelled"""
    return [t for t in range(D) if t not in (i, j) and entry(N, D, r, c, i, j, t) == 1]


def main():
    import threadpoolctl
    print([(d['internal_api'], d.get('version'), d.get('architecture')) for d in threadpoolctl.threadpool_info()])
    for N, D in ((256, 512), (256, 768), (256, 1024), (3000, 1024), (256, 1000), (3000, 1016), (256, 200)):
        print('N %d D %d: K-block boundaries %s' % (N, D, block_bounds(N, D)))
    s = sequential(256, 1024, 0, 16)
    print('D 1024, (i, j) = (0, 16): t joining after the cancellation: %d..%d (one chain, no lanes)' % (s[0], s[-1]))
    rng = np.random.default_rng(11)
    ok = tot = 0
    for N, D in ((300, 512), (200, 1024), (150, 768), (120, 1000), (90, 200), (64, 37)):
        X = rng.normal(0, 1, (N, D)).astype(np.float32)
        X[N // 2] = X[1] * np.float32(1.5)
        ok += np.array_equal(og.cosine_lower(X), og.cosine_lower_sklearn(X))
        tot += 1
    print('restatement == sklearn on every entry: %d of %d shapes' % (ok, tot))


if __name__ == '__main__':
    main()

"""Measure the float32 summation orders behind sklearn's K-means E-step in this container
(survey container; the goldens come from here) and check the restatement in oracle/kmeans.py
(estep_distances, einsum_sq), which the device kernel k_estep follows.

_update_chunk_dense (sklearn/cluster/_k_means_lloyd.pyx:168-215) computes, per 256-row chunk,
pd = row_norms(C, squared=True) (= np.einsum('ij,ij->i', C, C)) and then
_gemm(RowMajor, NoTrans, Trans, m, k, D, -2, X, D, C, D, 1, pd, k) -> scipy's OpenBLAS sgemm.

1. Absorption probes reveal a reduction tree: put x*c = 2^30 at position i, -2^30 at j and 1 at t;
   the result is 1 iff i and j cancel before t joins either of them.
2. The restated orders are then checked bit for bit against the libraries on random data.

    python scripts/sklearn_order.py
"""
import os
import sys

import numpy as np
from scipy.linalg import blas

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'video-to-faces_amd')]
from oracle.kmeans import _chunk_dist, einsum_sq  # noqa: E402

B = np.float32(2.0 ** 30)


def sk_gemm(X, C, csq):
    """the exact call _update_chunk_dense makes (RowMajor NoTrans/Trans -> Fortran 'T', 'N')"""
    pd = np.ascontiguousarray(np.broadcast_to(csq, (X.shape[0], C.shape[0])))
    return np.asarray(blas.sgemm(np.float32(-2.0), C.T, X.T, beta=1.0, c=pd.T, trans_a=1, trans_b=0)).T


def ranges(ts):
    out = []
    for t in ts:
        if out and t == out[-1][1] + 1:
            out[-1][1] = t
        else:
            out.append([t, t])
    return out


def probe_gemm(m, k, D, i, j, row=0, col=0):
    ones = []
    for t in range(D):
        if t in (i, j):
            continue
        X = np.zeros((m, D), np.float32)
        C = np.zeros((k, D), np.float32)
        for p, v in ((i, B), (j, -B), (t, 1)):
            X[row, p], C[col, p] = v, 1
        if round(float(sk_gemm(X, C, np.zeros(k, np.float32))[row, col]) / -2) == 1:
            ones.append(t)
    return ranges(ones)


def probe_einsum(D, i, j):
    ones = []
    for t in range(D):
        if t in (i, j):
            continue
        a = np.zeros((1, D), np.float32)
        b = np.zeros((1, D), np.float32)
        for p, v in ((i, B), (j, -B), (t, 1)):
            a[0, p], b[0, p] = v, 1
        if int(np.einsum('ij,ij->i', a, b)[0]) == 1:
            ones.append(t)
    return ranges(ones)


def main():
    print('einsum, D=64, (i, j) = (0, 1):', probe_einsum(64, 0, 1)[:6], '(lanes d mod 4, (l0+l1)+(l2+l3))')
    print('einsum, D=64, (i, j) = (0, 4):', probe_einsum(64, 0, 4)[:6], '(elements 12..15, 8..11, 4..7, 0..3)')
    print('sgemm blocked, m=256 k=10 D=1024, (500, 501):', probe_gemm(256, 10, 1024, 500, 501, 1, 0)[:3],
          '(K block boundary at 448)')
    print('sgemm small, m=7 k=2 D=1024, (0, 1):', probe_gemm(7, 2, 1024, 0, 1)[:3], '(16 lanes, adjacent pairs)')
    print('sgemm small, m=7 k=2 D=1024, (0, 16):', probe_gemm(7, 2, 1024, 0, 16)[:3], '(sequential per lane)')
    rng = np.random.default_rng(7)
    bad = tot = 0
    for D in (1024, 512, 768):
        C = rng.normal(0, 1, (64, D)).astype(np.float32)
        assert np.array_equal(einsum_sq(C), np.einsum('ij,ij->i', C, C))
        for k in range(2, 17):
            for m in (256, 255, 187, 128, 100, 50, 33, 16, 13, 9, 5, 2, 1):
                X = rng.normal(0, 1, (m, D)).astype(np.float32)
                C = rng.normal(0, 1, (k, D)).astype(np.float32)
                csq = einsum_sq(C)
                n = int((sk_gemm(X, C, csq) != _chunk_dist(X, C, csq)).sum())
                bad += n > 0
                tot += 1
                if n:
                    print('MISMATCH D', D, 'k', k, 'm', m, n)
    print('einsum restatement exact; E-step chunks exact: %d of %d shapes' % (tot - bad, tot))


if __name__ == '__main__':
    main()

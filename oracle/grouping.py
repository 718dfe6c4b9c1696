"""ORACLE — TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline leg).

Restatement of the grouping math the reference delegates to sklearn (sklearn 1.7.2 is
present in this image and on the GPU box; it is the reference's own unpinned dependency,
requirements.txt:5): dupes.py:60-65 and grouping.py:50-53.

cosine_dedupe / cosine_distances_exact: the C restatement (grouping_oracle.c) of
sklearn cosine_distances in the bits of numpy 2.2's einsum and OpenBLAS 0.3.29's SkylakeX
ssyrk (dedupe) and sgemm / sgemv / sdot (classify_distances_exact), pinned bit for bit against sklearn itself in the survey container
(tests/test_oracle.py::test_cosine_restatement_vs_sklearn, the grouping / scale goldens).  It
does not depend on the host's BLAS, so the GPU box (another CPU) checks against the same
bits.  cosine_lower_sklearn calls sklearn directly (used to pin the restatement here).
"""
import ctypes

import numpy as np
import sklearn.metrics

from oracle.nms import _lib


def _call(fn, X, *outs):
    X = np.ascontiguousarray(X, np.float32)
    fn(X.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(X.shape[0]), ctypes.c_int64(X.shape[1]),
       *[o.ctypes.data_as(ctypes.c_void_p) for o in outs])


def cosine_dedupe(X):
    """dupes.py:60-64: (mins, inds) of cosine_distances(X) + (1 - tri(k=-1)) * 10000."""
    n = X.shape[0]
    mins, inds = np.empty(n, np.float32), np.empty(n, np.int64)
    if n:
        _call(_lib().ora_cos_dedupe, X, mins, inds)
    return mins, inds


def cosine_distances_exact(X):
    """sklearn.metrics.pairwise.cosine_distances(X) (Y = X) in the reference's bits."""
    n = X.shape[0]
    out = np.empty((n, n), np.float32)
    if n:
        _call(_lib().ora_cos_distances, X, out)
    return out


def cosine_lower_sklearn(X):
    """dupes.py:60-62 with sklearn itself: cosine_distances + (1 - tri(k=-1)) * 10000."""
    D = sklearn.metrics.pairwise.cosine_distances(X)
    D += (1 - np.tri(X.shape[0], k=-1).astype(D.dtype)) * 10000
    return D


def cosine_lower(X):
    """the masked matrix of dupes.py:60-62 from the restatement"""
    D = cosine_distances_exact(X)
    D += (1 - np.tri(X.shape[0], k=-1).astype(D.dtype)) * 10000
    return D


def classify(X, R):
    D = sklearn.metrics.pairwise.cosine_distances(X, R)
    return D.min(axis=1), D.argmin(axis=1)


def classify_distances_exact(X, R):
    """grouping.py:51 cosine_distances(X, R) in the reference's bits (grouping_oracle.c: numpy's
    OpenBLAS sgemm blocked / small-matrix, sgemv 4x4 / 4x2 / 4x1 kernels over 8 threads, sdot)."""
    X = np.ascontiguousarray(X, np.float32)
    R = np.ascontiguousarray(R, np.float32)
    out = np.empty((X.shape[0], R.shape[0]), np.float32)
    if X.shape[0]:
        _lib().ora_cos_classify_dist(X.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(X.shape[0]),
                                     R.ctypes.data_as(ctypes.c_void_p), ctypes.c_int64(R.shape[0]),
                                     ctypes.c_int64(X.shape[1]), ctypes.c_int(0), out.ctypes.data_as(ctypes.c_void_p))
    return out

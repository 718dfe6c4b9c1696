"""ORACLE — TEST INFRASTRUCTURE ONLY (tests/, smoke(), bench.py cpu_baseline leg).

Restatement of the grouping math the reference delegates to sklearn (sklearn 1.7.2 is
present in this image and on the GPU box; it is the reference's own unpinned dependency,
requirements.txt:5): dupes.py:60-65 and grouping.py:50-53.
"""
import numpy as np
import sklearn.metrics


def cosine_lower(X):
    """dupes.py:60-62: cosine_distances + (1 - tri(k=-1)) * 10000."""
    D = sklearn.metrics.pairwise.cosine_distances(X)
    D += (1 - np.tri(X.shape[0], k=-1).astype(D.dtype)) * 10000
    return D


def cosine_dedupe(X):
    D = cosine_lower(X)
    return D.min(axis=1), D.argmin(axis=1)


def classify(X, R):
    D = sklearn.metrics.pairwise.cosine_distances(X, R)
    return D.min(axis=1), D.argmin(axis=1)

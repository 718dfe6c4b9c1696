"""GPU parity: fused cosine dedupe / classify vs sklearn goldens (dupes.py:51-68, grouping.py:50-66)."""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def g():
    return np.load(os.path.join(GOLDEN, 'grouping.npz'))


def test_cosine_dedupe_vs_golden(g):
    from videotofaces import dupes
    mins, inds = dupes.cosine_dedupe_device(torch.from_numpy(g['X']).cuda())
    np.testing.assert_allclose(mins, g['dedupe_mins'], atol=1e-5, rtol=0)
    np.testing.assert_array_equal(inds, g['dedupe_inds'])
    keep = np.nonzero(~(mins <= 0.25))[0]
    np.testing.assert_array_equal(keep, g['dedupe_keep'])


def test_cosine_dedupe_large_vs_oracle():
    from videotofaces import dupes
    from oracle import grouping as og
    rng = np.random.default_rng(5)
    X = rng.normal(0, 1, (3000, 512)).astype(np.float32)
    X[1500:1510] = X[10:20] + 1e-3
    X[7] = 0  # zero-norm row (sklearn normalize maps the norm to 1)
    mins, inds = dupes.cosine_dedupe_device(torch.from_numpy(X).cuda())
    rm, ri = og.cosine_dedupe(X)
    np.testing.assert_allclose(mins, rm, atol=1e-5)
    D = og.cosine_lower(X)
    rows = np.nonzero(inds != ri)[0]
    # argmin may differ only where two earlier faces are within fp32 GEMM rounding
    assert np.all(np.abs(D[rows, inds[rows]] - D[rows, ri[rows]]) < 1e-5)


def test_classify_vs_golden(g):
    from videotofaces import grouping
    inds, classes = grouping.classify(g['X'], g['classify_R'], ['a', 'b', 'c'], 0.9, False, [], None)
    np.testing.assert_array_equal(inds, g['classify_inds'])
    assert classes == ['a', 'b', 'c', 'other']

"""GPU parity: hash dedupe (src/videotofaces/dupes.py:11-65) on libvtf_hip.so.

Bit-exact integer work: the Hamming row-min / first-argmin and the kept set equal the
reference's remove_dupes_overall('hash') (tests/golden/dupes.npz); the GPU average hash equals
the oracle's restatement of cv2 cvtColor + INTER_LINEAR resize (cv2 absent: that step is
parity-unpinned against OpenCV itself).
"""
import os

import numpy as np
import pytest
import torch

from conftest import GOLDEN

pytestmark = pytest.mark.gpu


def test_hamming_vs_golden():
    from videotofaces.dupes import hamming_lower
    g = np.load(os.path.join(GOLDEN, 'dupes.npz'))
    mins, inds = hamming_lower(g['X'])
    np.testing.assert_array_equal(mins, g['mins'].astype(np.int32))
    np.testing.assert_array_equal(inds, g['inds'])


def test_remove_dupes_overall_hash_vs_golden():
    from videotofaces.dupes import remove_dupes_overall
    g = np.load(os.path.join(GOLDEN, 'dupes.npz'))
    names = ['f%05d.jpg' % i for i in range(g['X'].shape[0])]
    X, goods = remove_dupes_overall(g['X'].copy(), names, ('hash', 8, False, None))
    assert [int(n[1:6]) for n in goods] == g['keep'].tolist()
    assert X.shape[0] == len(goods)


def test_hamming_large_vs_numpy():
    from videotofaces.dupes import hamming_lower
    rng = np.random.default_rng(4)
    n = 5000
    h = rng.integers(0, 2**63, n, dtype=np.int64).view(np.uint64)
    h[100:200] = h[:100] ^ np.uint64(1)  # planted near-duplicates
    mins, inds = hamming_lower(h)
    hb = ((h[:, None] >> np.arange(64, dtype=np.uint64)) & np.uint64(1)).astype(np.uint8)
    for i in (0, 1, 150, 4999):
        d = (hb[:i] != hb[i]).sum(1)
        if i == 0:
            assert mins[0] == 10000 and inds[0] == 0
        else:
            assert mins[i] == d.min() and inds[i] == d.argmin()


def test_ahash_vs_oracle():
    from oracle import dupes as od
    from videotofaces import synth
    from videotofaces.dupes import ahash_crops, unpack_hash
    fr = synth.make_frames(2, 180, 320, seed=6)
    rng = np.random.default_rng(5)
    crops = [[0, 10, 20, 26, 36], [1, 5, 5, 13, 13], [0, 0, 0, 320, 180], [1, 100, 50, 101, 51]]
    for _ in range(60):
        f = int(rng.integers(0, 2))
        x1, y1 = int(rng.integers(0, 300)), int(rng.integers(0, 160))
        x2, y2 = int(rng.integers(x1 + 1, 321)), int(rng.integers(y1 + 1, 181))
        crops.append([f, x1, y1, x2, y2])
    got = ahash_crops(torch.from_numpy(fr).cuda(), np.array(crops))
    for c, h in zip(crops, got):
        f, x1, y1, x2, y2 = c
        np.testing.assert_array_equal(unpack_hash(h), od.ahash(fr[f, y1:y2, x1:x2]), err_msg=str(c))

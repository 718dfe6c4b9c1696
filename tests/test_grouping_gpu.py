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
    np.testing.assert_array_equal(mins, g['dedupe_mins'])
    np.testing.assert_array_equal(inds, g['dedupe_inds'])
    keep = np.nonzero(~(mins <= 0.25))[0]
    np.testing.assert_array_equal(keep, g['dedupe_keep'])


@pytest.mark.parametrize('D,valu', [(512, '0'), (512, '1'), (1000, '0'), (1024, '0')])
def test_cosine_dedupe_large_vs_oracle(D, valu, monkeypatch):
    """mins and argmins bit-exact vs the pinned restatement of sklearn's bits
    (oracle/grouping_oracle.c), both kernel forms: the fp32-MFMA tiles (K blocks on 4-steps) and
    the VALU fmaf tiles (VTF_COS_VALU=1; D = 1000 has a K block ending at 724 and also runs the
    MFMA form since 724 % 4 == 0)."""
    from videotofaces import dupes
    from oracle import grouping as og
    monkeypatch.setenv('VTF_COS_VALU', valu)
    rng = np.random.default_rng(5)
    X = rng.normal(0, 1, (3000, D)).astype(np.float32)
    X[1500:1510] = X[10:20] + 1e-3
    X[2000:2003] = X[100]  # exact ties: the first index wins, as numpy's argmin
    X[7] = 0  # zero-norm row (sklearn normalize maps the norm to 1)
    mins, inds = dupes.cosine_dedupe_device(torch.from_numpy(X).cuda())
    rm, ri = og.cosine_dedupe(X)
    np.testing.assert_array_equal(mins, rm)
    np.testing.assert_array_equal(inds, ri)


def test_cosine_dedupe_row_ranges_join():
    """The row-range entry (vtf_cosine_dedupe_rows, used per rank by cosine_dedupe_sharded) over
    uneven shards of N = 1000 (not a multiple of 128) joins to the full-range result bit for bit;
    likewise the silhouette sweep over uneven row splits."""
    from videotofaces import dupes
    from videotofaces.kmeans import Grouper
    rng = np.random.default_rng(9)
    N = 1000
    X = rng.normal(0, 1, (N, 256)).astype(np.float32)
    X[600:650] = X[0:50] + 0.05
    Xd = torch.from_numpy(X).cuda()
    fm, fi = dupes.cosine_dedupe_rows(Xd, 0, N)
    for w in (2, 3, 5):
        b = dupes.dedupe_shards(N, w)
        parts = [dupes.cosine_dedupe_rows(Xd, b[r], b[r + 1]) for r in range(w)]
        np.testing.assert_array_equal(np.concatenate([p[0] for p in parts]), fm)
        np.testing.assert_array_equal(np.concatenate([p[1] for p in parts]), fi)
    gr = Grouper('cuda:0')
    lbs = [gr.kmeans(X, k) for k in (2, 5)]
    full = gr.silhouette_sweep(X, lbs, 0, N)
    for cuts in ((0, 333, 1000), (0, 1, 517, 999, 1000)):
        parts = [gr.silhouette_sweep(X, lbs, lo, hi) for lo, hi in zip(cuts[:-1], cuts[1:])]
        for i in range(len(lbs)):
            np.testing.assert_array_equal(np.concatenate([p[i] for p in parts]), full[i])


def test_classify_vs_golden(g):
    from videotofaces import grouping
    inds, classes = grouping.classify(g['X'], g['classify_R'], ['a', 'b', 'c'], 0.9, False, [], None)
    np.testing.assert_array_equal(inds, g['classify_inds'])
    assert classes == ['a', 'b', 'c', 'other']


def _classify_cases():
    import sys
    sys.path.insert(0, GOLDEN)
    from make_golden import CLASSIFY_CASES
    return CLASSIFY_CASES


@pytest.mark.parametrize('case', _classify_cases(), ids=lambda c: c[0])
def test_classify_sklearn_bits_vs_golden(case, tmp_path):
    """classify (grouping.py:50-66) in sklearn's exact bits, every matmul form sklearn reaches:
    the planted 10k x 8 set (a third of the rows within +-2e-6 of the 'other' threshold, 41 of
    them exactly on it; a third near-tied between two classes, 405 exact ties) and the small /
    gemv (1 and 8 BLAS threads) / vector-matrix / dot shapes.  Assigned indices (incl. 'other'),
    the full distance matrix and the log_classification.csv text equal the reference's."""
    import hashlib
    from videotofaces import grouping, synth
    name, N, C, D, thr, seed = case
    g = np.load(os.path.join(GOLDEN, 'classify.npz'))
    X, R = synth.classify_set(N, C, D, thr or 0.9, seed)
    assert hashlib.sha256(X.tobytes() + R.tobytes()).hexdigest() == str(g[name + '_x_sha'])
    np.testing.assert_array_equal(grouping.cosine_distances_device(X, R), g[name + '_dist'])
    os.makedirs(tmp_path / 'faces')
    paths = ['/x/face_%05d.jpg' % i for i in range(N)]
    inds, classes = grouping.classify(X, R, ['c%d' % i for i in range(C)], thr, True, paths, str(tmp_path))
    np.testing.assert_array_equal(inds, g[name + '_inds'])
    assert len(classes) == int(g[name + '_ncls'])
    csv = open(tmp_path / 'faces' / 'log_classification.csv').read()
    assert hashlib.sha256(csv.encode()).hexdigest() == str(g[name + '_csv_sha'])
    if name == 'planted':
        print('other %d, on the threshold %d' % (int((inds == C).sum()), int((g[name + '_dist'].min(1) == np.float32(thr)).sum())))


def test_classify_nan_rows_vs_oracle():
    """a NaN row: numpy's min is NaN and argmin the first NaN (the reference's dist.min /
    argmin); zero rows normalise with norm 1 (distance 1)"""
    from videotofaces import grouping, synth
    from oracle import grouping as og
    X, R = synth.classify_set(64, 4, 512, 0.9, seed=11)
    X[5, 7] = np.nan
    X[9] = 0
    ref = og.classify_distances_exact(X, R)
    got = grouping.cosine_distances_device(X, R)
    np.testing.assert_array_equal(got, ref)
    mins, inds = grouping.cosine_classify_device(X, R)
    np.testing.assert_array_equal(mins, ref.min(1))
    np.testing.assert_array_equal(inds, ref.argmin(1))


def test_wide_rows_vs_oracle():
    """Rows wider than k_row_normalize's LDS staging (D > 4096: the four staged rows would pass the
    64 KB dynamic-LDS default) take the global-memory form, same bits: dedupe minima / argmins and
    the classify distance matrix vs the restatement (oracle/grouping_oracle.c)."""
    from videotofaces import dupes, grouping, synth
    from oracle import grouping as og
    rng = np.random.default_rng(21)
    X = rng.normal(0, 1, (400, 4160)).astype(np.float32)
    X[300:310] = X[0:10] + 1e-3
    mins, inds = dupes.cosine_dedupe_device(torch.from_numpy(X).cuda())
    rm, ri = og.cosine_dedupe(X)
    np.testing.assert_array_equal(mins, rm)
    np.testing.assert_array_equal(inds, ri)
    Xc, R = synth.classify_set(64, 4, 4160, 0.9, seed=3)
    np.testing.assert_array_equal(grouping.cosine_distances_device(Xc, R), og.classify_distances_exact(Xc, R))


@pytest.fixture(scope='module')
def km():
    from videotofaces import synth
    return np.load(os.path.join(GOLDEN, 'kmeans.npz')), synth.planted_clusters()


def test_kmeans_labels_vs_sklearn(km):
    """KMeans(k, random_state=0, n_init='auto') labels for k = 2..16 (N=2000, D=512):
    bit-exact integer labels against sklearn."""
    from videotofaces.kmeans import Grouper
    g, X = km
    gr = Grouper('cuda:0')
    prep = gr.prepare(X)
    for i, k in enumerate(g['k']):
        np.testing.assert_array_equal(gr.kmeans(X, int(k), prep=prep), g['labels'][i], err_msg='k=%d' % k)


def test_kmeans_small_golden(g):
    """grouping.npz: the reference-path sweep (k=2..9) on the deduped 600-row set."""
    from videotofaces import dupes
    from videotofaces.kmeans import Grouper
    mins, _ = dupes.cosine_dedupe_device(torch.from_numpy(g['X']).cuda())
    Xk = g['X'][~(mins <= 0.25)]
    gr = Grouper('cuda:0')
    for i, k in enumerate(g['kmeans_k']):
        lb = gr.kmeans(Xk, int(k))
        np.testing.assert_array_equal(lb, g['kmeans_labels'][i], err_msg='k=%d' % k)
        s1 = gr.silhouette_score(Xk, lb)
        s2 = gr.calinski_harabasz_score(Xk, lb)
        s3 = gr.davies_bouldin_score(Xk, lb)
        np.testing.assert_allclose([s1, s2, s3], g['cluster_scores'][i], rtol=1e-5)


def test_silhouette_and_scores_vs_sklearn(km):
    from videotofaces.kmeans import Grouper
    g, X = km
    gr = Grouper('cuda:0')
    sil = gr.silhouette_samples(X, g['labels'][6])
    np.testing.assert_allclose(sil, g['sil_k8'], rtol=0, atol=2e-7)
    print('silhouette samples exact:', np.array_equal(sil, g['sil_k8']))
    for i in (0, 6, 14):
        lb = g['labels'][i]
        got = [gr.silhouette_score(X, lb), gr.calinski_harabasz_score(X, lb), gr.davies_bouldin_score(X, lb)]
        np.testing.assert_allclose(got, g['scores'][i], rtol=1e-5)


def test_cluster_sweep_best_k(km):
    from videotofaces.grouping import cluster_sweep
    g, X = km
    ks = [int(k) for k in g['k']]
    labels, scores = cluster_sweep(X, ks, 0)
    best = max(scores, key=lambda x: x[1])[0]
    assert best == ks[int(np.argmax(g['scores'][:, 0]))]
    for i in range(len(ks)):
        np.testing.assert_array_equal(labels[i], g['labels'][i])


@pytest.fixture(scope='module')
def scale():
    """tests/golden/scale.npz (make_golden.py gen_scale): 30k realistic embeddings regenerated
    from the chain's ViT-L rows, checked by hash."""
    import hashlib
    import json
    from videotofaces import synth
    g = np.load(os.path.join(GOLDEN, 'scale.npz'))
    c = json.loads(str(g['params_json']))
    X = synth.video_embeddings(np.load(os.path.join(GOLDEN, 'chain.npz'))['X'], c['n'], seed=c['seed'])
    assert hashlib.sha256(X.tobytes()).digest() == g['X_sha256'].tobytes()
    return g, X


def test_scale_dedupe_30k(scale):
    """remove_dupes_overall('enc') at N = 30k on realistic embeddings (D = 1024): mins, argmins
    and the keep set bit-exact vs sklearn's own output (the golden)."""
    import time
    from videotofaces import dupes
    g, X = scale
    Xd = torch.from_numpy(X).cuda()
    dupes.cosine_dedupe_device(Xd)
    torch.cuda.synchronize()
    t = time.time()
    mins, inds = dupes.cosine_dedupe_device(Xd)
    dt = time.time() - t
    np.testing.assert_array_equal(mins, g['dedupe_mins'])
    np.testing.assert_array_equal(inds, g['dedupe_inds'])
    np.testing.assert_array_equal(np.nonzero(~(mins <= 0.25))[0], g['dedupe_keep'])
    print('kept %d of %d, exact; %.1f ms' % (int((~(mins <= 0.25)).sum()), len(X), dt * 1e3))


def test_scale_kmeans_sweep_20k(scale):
    """cluster_faces' sweep (grouping.py:97-107) on the ~20k deduped rows, D = 1024, k = 2..16:
    labels bit-exact vs sklearn (1 OpenMP thread, deterministic; the golden records where
    sklearn with every core differs from itself -- those rows are the only ones allowed to
    differ), silhouette / CH / DB within rtol 1e-5."""
    from videotofaces.grouping import cluster_sweep
    g, X = scale
    Xk = X[g['dedupe_keep']]
    ks = [int(k) for k in g['k']]
    labels, scores = cluster_sweep(Xk, ks, 0)
    for i, k in enumerate(ks):
        bad = np.nonzero(labels[i] != g['labels'][i])[0]
        sk_self = np.nonzero(g['labels'][i] != g['labels_mt'][i])[0]
        assert np.isin(bad, sk_self).all(), 'k=%d: %d rows differ from sklearn (sklearn self-disagreement %d)' % (
            k, len(bad), len(sk_self))
    np.testing.assert_allclose(np.array([s[1:] for s in scores]), g['scores'], rtol=1e-5)
    print('N', len(Xk), 'best k', max(scores, key=lambda x: x[1])[0])


def test_sweep_200k_rows_no_nxn():
    """The k = 2..16 sweep at N = 200k, D = 1024 in one process (an N x N fp32 matrix would be
    160 GB): KMeans fits, the one-pass silhouette over the distance rows, CH / DB.  A 256-row
    sample of the silhouette is checked against a float64 numpy restatement (distances of those
    rows to all N; tolerance 1e-5, the fp32 rounding of the per-cluster sums), and the device
    memory in use after the sweep stays O(N D)."""
    import time
    from videotofaces import synth
    from videotofaces.grouping import cluster_sweep
    from videotofaces.kmeans import Grouper
    basis = np.load(os.path.join(GOLDEN, 'chain.npz'))['X']
    X = synth.video_embeddings(basis, 200000, seed=5)
    ks = list(range(2, 17))
    t = time.time()
    labels, scores = cluster_sweep(X, ks, 0)
    dt = time.time() - t
    free, total = torch.cuda.mem_get_info()
    print('sweep N=200k: %.1f s, device memory in use %.1f GB, best k %d'
          % (dt, (total - free) / 1e9, max(scores, key=lambda s: s[1])[0]))
    assert (total - free) < 40e9
    for lb, k in zip(labels, ks):
        assert lb.min() == 0 and lb.max() == k - 1
    assert all(np.isfinite(s[1:]).all() for s in scores)
    rows = np.random.default_rng(0).choice(len(X), 256, replace=False)
    lb = labels[6]
    sil = Grouper('cuda:0').silhouette_sweep(X, [lb], 0, len(X))[0][rows]
    X64 = X.astype(np.float64)
    n2 = (X64 * X64).sum(1)
    d = np.sqrt(np.maximum((n2[rows, None] - 2 * X64[rows] @ X64.T + n2[None, :]).astype(np.float32), 0))
    d[np.arange(len(rows)), rows] = 0
    freq = np.bincount(lb)
    cd = np.stack([d[:, lb == c].astype(np.float64).sum(1) for c in range(len(freq))], 1).astype(np.float32)
    own = lb[rows]
    a = cd[np.arange(len(rows)), own] / (freq[own] - 1)
    cd[np.arange(len(rows)), own] = np.inf
    b = (cd / freq).min(1)
    ref = (b - a) / np.maximum(a, b)
    np.testing.assert_allclose(sil, ref, rtol=0, atol=1e-5)

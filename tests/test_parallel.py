"""CPU: multi-process (gloo, world_size 2) coverage of the frame sharding and the rank-ordered
all-gather-v of embeddings used by bench.py / the N>1 path."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def test_shard_batches_cover_and_align():
    from videotofaces.parallel import shard_batches
    for n, bs, world in [(100, 16, 2), (10000, 16, 8), (5, 4, 3), (0, 4, 2), (33, 16, 4)]:
        ranges = [shard_batches(n, bs, r, world) for r in range(world)]
        assert ranges[0][0] == 0 and ranges[-1][1] == n
        for (a, b), (c, d) in zip(ranges, ranges[1:]):
            assert b == c
        for a, b in ranges:
            assert (a % bs == 0 or a == n) and (b % bs == 0 or b == n)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, 'video-to-faces_amd')]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from videotofaces.parallel import all_gather_rows, shard_batches
    n_frames, bs = 70, 16
    lo, hi = shard_batches(n_frames, bs, rank, world)
    # a stand-in for per-frame embeddings: row = [frame index, face index]; frame f has f % 3 faces
    rows = [[f, k] for f in range(lo, hi) for k in range(f % 3)]
    local = torch.tensor(rows, dtype=torch.float32).reshape(-1, 2)
    out = all_gather_rows(local)
    q.put((rank, out.tolist()))
    dist.destroy_process_group()


def test_all_gather_rows_rank_order_gloo():
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=120) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    expect = [[f, k] for f in range(70) for k in range(f % 3)]
    for r in range(world):
        assert res[r] == expect


def _sweep_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, 'video-to-faces_amd')]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from oracle.kmeans import CpuGrouper
    from videotofaces import synth
    from videotofaces.grouping import cluster_sweep
    X = synth.planted_clusters(N=400, D=32)
    done = []

    class Spy(CpuGrouper):
        def kmeans(self, X, k, **kw):
            done.append(k)
            return super().kmeans(X, k, **kw)

        def silhouette_sweep(self, X, label_sets, lo=0, hi=None):
            done.append(('rows', lo, hi))
            return super().silhouette_sweep(X, label_sets, lo, hi)
    labels, scores = cluster_sweep(X, [2, 3, 4, 5, 6], 0, Spy(), sharded=True)
    q.put((rank, done, [lb.tolist() for lb in labels], scores))
    dist.destroy_process_group()


def test_cluster_sweep_sharded_gloo():
    """The sweep split across 2 ranks: KMeans fits by k (i % world), the
    silhouette by row ranges, CH/DB by k; every rank ends with labels and scores identical to
    the one-process sweep."""
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_sweep_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {r: (d, lb, sc) for r, d, lb, sc in (q.get(timeout=180) for _ in range(world))}
    for p in ps:
        p.join(timeout=60)
    assert res[0][0] == [2, 4, 6, ('rows', 0, 200)] and res[1][0] == [3, 5, ('rows', 200, 400)]
    assert res[0][1] == res[1][1] and res[0][2] == res[1][2]
    from oracle.kmeans import CpuGrouper
    from videotofaces import synth
    from videotofaces.grouping import cluster_sweep
    X = synth.planted_clusters(N=400, D=32)
    labels, scores = cluster_sweep(X, [2, 3, 4, 5, 6], 0, CpuGrouper())
    assert res[0][1] == [lb.tolist() for lb in labels]
    assert res[0][2] == scores


def _dedupe_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, 'video-to-faces_amd')]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    import numpy as np
    from oracle import grouping as og
    from videotofaces.dupes import cosine_dedupe_sharded
    X = np.random.default_rng(3).normal(0, 1, (1000, 16)).astype(np.float32)
    rm, ri = og.cosine_dedupe(X)
    seen = []

    def rows_fn(lo, hi):
        seen.append((lo, hi))
        return rm[lo:hi], ri[lo:hi]
    mins, inds = cosine_dedupe_sharded(X, rows_fn)
    q.put((rank, seen, mins.tolist(), inds.tolist()))
    dist.destroy_process_group()


def test_cosine_dedupe_sharded_gloo():
    """The lower-triangle dedupe row-block sharded over 3 ranks (128-aligned, balanced by area)
    and all-gathered: every rank ends with the full (min, argmin) of every row."""
    import numpy as np
    from oracle import grouping as og
    from videotofaces.dupes import dedupe_shards
    world = 3
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_dedupe_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {r: rest for r, *rest in (q.get(timeout=180) for _ in range(world))}
    for p in ps:
        p.join(timeout=60)
    b = dedupe_shards(1000, world)
    assert [res[r][0] for r in range(world)] == [[(b[r], b[r + 1])] for r in range(world)]
    assert all(x % 128 == 0 for x in b[:-1]) and b[-1] == 1000
    X = np.random.default_rng(3).normal(0, 1, (1000, 16)).astype(np.float32)
    rm, ri = og.cosine_dedupe(X)
    for r in range(world):
        assert res[r][1] == rm.tolist() and res[r][2] == ri.tolist()
    # area balance: each shard holds roughly 1/world of the lower triangle's tile pairs
    nt = [(x + 127) // 128 for x in b]
    pairs = [nt[r + 1] * (nt[r + 1] + 1) // 2 - nt[r] * (nt[r] + 1) // 2 for r in range(world)]
    assert max(pairs) <= 2 * min(pairs) + 8


def _mismatch_worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [root, os.path.join(root, 'video-to-faces_amd')]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port))
    dist.init_process_group('gloo', rank=rank, world_size=world)
    from oracle.kmeans import CpuGrouper
    from videotofaces import synth
    from videotofaces.grouping import cluster_sweep
    X = synth.planted_clusters(N=100 + rank, D=8)  # ranks disagree
    try:
        cluster_sweep(X, [2, 3], 0, CpuGrouper(), sharded=True)
        q.put((rank, 'no error'))
    except ValueError as e:
        q.put((rank, str(e)))
    dist.destroy_process_group()


def test_sharded_sweep_refuses_different_inputs_gloo():
    """A sharded grouping step whose ranks hold different embeddings raises on every rank
    instead of stitching shards of different inputs together."""
    world = 2
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_mismatch_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=180) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert all('ranks hold different inputs' in res[r] for r in range(world)), res

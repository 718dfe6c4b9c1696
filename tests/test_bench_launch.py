"""CPU: bench.py's multi-GPU plumbing without a GPU.

* --gpus N without a torchrun environment re-launches itself through torch.distributed.run
  (checked on the command it builds); a WORLD_SIZE that disagrees with --gpus is refused
  before anything touches a GPU;
* measure() -- barrier + sync brackets, max-over-ranks time, summed faces, rank-ordered
  all-gather-v of embeddings -- on a world-size-2 gloo group with a stand-in pipeline whose
  "embeddings" are (frame, face) rows: the gathered rows must equal the world-1 run's.
"""
import os
import socket
import subprocess
import sys

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
N_FRAMES, DET_BS = 100, 8


def test_presets_and_overrides():
    import bench
    a = bench.parse([])
    assert (a.config, a.det_model, a.enc_model, a.det_batch, a.enc_batch, a.H) == ('c2', 'mtcnn', 'facenet', 16, 128, 720)
    a = bench.parse(['--config', 'c5'])
    assert (a.det_model, a.enc_model, a.det_batch, a.H, a.W, a.grouping, a.enc_precision) == \
        ('yolo', 'vit_l', 32, 1080, 1920, True, 'f16x')
    a = bench.parse(['--config', 'c4'])
    assert (a.det_model, a.enc_model, a.enc_batch) == ('none', 'vit_l', 128)
    a = bench.parse(['--config', 'c3', '--det-batch', '8', '--enc-precision', 'fp32'])
    assert (a.det_model, a.det_batch, a.enc_precision, a.det_min_size) == ('yolo', 8, 'fp32', 50)


def test_spawn_command():
    import bench
    cmd = bench.spawn_command(8, ['--gpus', '8', '--steps', '5'], 29511)
    assert cmd[:3] == [sys.executable, '-m', 'torch.distributed.run']
    assert '--nproc-per-node' in cmd and cmd[cmd.index('--nproc-per-node') + 1] == '8'
    assert cmd[cmd.index('--master-addr') + 1] == '127.0.0.1'
    assert cmd[-4:] == ['--gpus', '8', '--steps', '5'] and cmd[-5].endswith('bench.py')


def test_world_size_mismatch_is_refused():
    env = dict(os.environ, WORLD_SIZE='1', RANK='0', LOCAL_RANK='0')
    r = subprocess.run([sys.executable, os.path.join(ROOT, 'bench.py'), '--gpus', '2'], env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 2 and 'WORLD_SIZE' in r.stderr


class StubPipeline:
    """Stand-in for the GPU pipelines: step i of this rank encodes det-batch i of its shard;
    frame f yields f % 3 "faces" whose embedding row is (f, face index)."""

    def __init__(self, rank, world):
        from videotofaces.parallel import shard_batches
        self.lo, self.hi = shard_batches(N_FRAMES, DET_BS, rank, world)
        self.D = 2

    def steps(self):
        return -(-(self.hi - self.lo) // DET_BS)

    def run(self, first, n):
        stats, parts = [], []
        for i in range(first, first + n):
            f0 = self.lo + i * DET_BS
            rows = [[f, k] for f in range(f0, min(f0 + DET_BS, self.hi)) for k in range(f % 3)]
            stats.append(len(rows))
            parts.append(torch.tensor(rows, dtype=torch.float32).reshape(-1, 2))
        return stats, parts


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, 'video-to-faces_amd')]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import bench
    ctx = bench.Ctx('gloo', device=torch.device('cpu'))
    pipe = StubPipeline(rank, world)
    # equal step counts across ranks (the bench times the same K on every rank)
    faces, el, gathered, stats = bench.measure(pipe, pipe.steps(), 0, ctx)
    q.put((rank, ctx.world, faces, el, gathered.tolist()))
    ctx.close()


def test_measure_world2_gloo_matches_world1():
    import bench
    pipe1 = StubPipeline(0, 1)
    ctx1 = bench.Ctx('gloo', device=torch.device('cpu'))
    assert ctx1.world == 1
    f1, _, g1, _ = bench.measure(pipe1, pipe1.steps(), 0, ctx1)
    world = 2
    mpc = mp.get_context('spawn')
    q = mpc.Queue()
    port = _free_port()
    ps = [mpc.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {r: (w, f, e, g) for r, w, f, e, g in (q.get(timeout=180) for _ in range(world))}
    for p in ps:
        p.join(timeout=60)
    assert all(res[r][0] == 2 for r in range(world))
    assert res[0][1] == res[1][1] == f1 == g1.shape[0]
    assert res[0][2] == res[1][2]  # max over ranks
    assert res[0][3] == res[1][3] == g1.tolist()


# ---- DetEncPipeline over one global frame sequence, with CPU stand-ins for the HIP models
H_, W_, BS_, STEPS_ = 48, 64, 4, 6


class StubDetector:
    """crops: per frame, the 8x8 cells whose green mean is above the frame's 80th percentile
    (at most 3, row-major); deterministic in the frame content"""

    def detect_crops(self, src, minsize, bp, off):
        out = []
        for f in range(src.shape[0]):
            g = src[f, :, :, 1].float().reshape(H_ // 8, 8, W_ // 8, 8).mean((1, 3))
            cells = torch.nonzero(g > torch.quantile(g, 0.8))[:3]
            for cy, cx in cells.tolist():
                out.append([off + f, cx * 8, cy * 8, cx * 8 + 16, cy * 8 + 16])
        return torch.tensor(out, dtype=torch.int32).reshape(-1, 5), None


class StubEncoder:
    dim = 12

    def encode_crops(self, frames, crops):
        rows = []
        for f, x1, y1, x2, y2 in crops.tolist():
            c = frames[f, y1:y2, x1:x2].float()
            rows.append(torch.cat([c.mean((0, 1)), c.std((0, 1)), c[::4, ::4].reshape(-1, 3).amax(0),
                                   c[:, :, 1].reshape(-1)[:3]]))
        return torch.stack(rows) if rows else torch.zeros((0, self.dim))


def _pipe_args():
    import bench
    a = bench.parse(['--config', 'c2', '--det-batch', str(BS_), '--pool', '0', '--lanes', '2', '--enc-batch', '5',
                     '--enc-model', 'vit_b'])
    a.H, a.W = H_, W_
    return a


def _pipeline_run(ctx):
    """frames of the rank's shard (rank_frames, pool 0: distinct frames from one global sequence)
    -> stand-in detector / encoder lanes -> measure (all-gather-v) -> grouping_leg (dedupe rows
    sharded + the k sweep sharded) with the oracle restatements as the device kernels"""
    import numpy as np
    import bench
    from oracle import grouping as og
    from oracle.kmeans import CpuGrouper
    a = _pipe_args()
    frames, offset, fnp = bench.rank_frames(a, ctx, STEPS_)
    pipe = bench.DetEncPipeline(a, ctx.device, frames, offset, fnp, StubDetector, StubEncoder)
    faces, _, X, _ = bench.measure(pipe, STEPS_, 0, ctx)
    Xh = X.numpy()
    rm, ri = og.cosine_dedupe(Xh)
    rec, mins, labels, scores = bench.grouping_leg(X, ctx, ctx.device, rows_fn=lambda lo, hi: (rm[lo:hi], ri[lo:hi]),
                                                   grouper=CpuGrouper())
    return faces, Xh.tolist(), np.asarray(mins).tolist(), [np.asarray(lb).tolist() for lb in labels], scores, rec


def _pipe_worker(rank, world, port, q):
    sys.path[:0] = [ROOT, os.path.join(ROOT, 'video-to-faces_amd')]
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import bench
    ctx = bench.Ctx('gloo', device=torch.device('cpu'))
    q.put((rank, _pipeline_run(ctx)))
    ctx.close()


def test_det_enc_pipeline_world2_matches_world1_gloo():
    """SURVEY.md §8e as bench.py runs it: each rank takes its whole det-batches of ONE global
    frame sequence (parallel.shard_batches), detects and encodes them on two lanes, the
    embeddings are all-gathered in frame order, then the dedupe and the k sweep run sharded.
    World 2 (gloo) gathers exactly the embeddings of world 1 over the same 2 x 6 det-batches and
    ends with the same dedupe minima, labels and scores."""
    import bench
    world = 2
    mpc = mp.get_context('spawn')
    q = mpc.Queue()
    port = _free_port()
    ps = [mpc.Process(target=_pipe_worker, args=(r, world, port, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict(q.get(timeout=300) for _ in range(world))
    for p in ps:
        p.join(timeout=60)
    assert res[0][:5] == res[1][:5]

    # world 1 over the same global sequence: the one rank takes all 2 x STEPS_ det-batches
    ctx1 = bench.Ctx('gloo', device=torch.device('cpu'))
    b2 = bench
    a = _pipe_args()
    frames, offset, fnp = b2.rank_frames(a, ctx1, world * STEPS_)
    pipe = b2.DetEncPipeline(a, ctx1.device, frames, offset, fnp, StubDetector, StubEncoder)
    faces1, _, X1, _ = b2.measure(pipe, world * STEPS_, 0, ctx1)
    assert res[0][0] == faces1 and res[0][1] == X1.numpy().tolist()
    assert len(res[0][1]) > 40
    import numpy as np
    from oracle import grouping as og
    from oracle.kmeans import CpuGrouper
    rm, ri = og.cosine_dedupe(X1.numpy())
    _, mins1, labels1, scores1 = b2.grouping_leg(X1, ctx1, ctx1.device, rows_fn=lambda lo, hi: (rm[lo:hi], ri[lo:hi]),
                                                 grouper=CpuGrouper())
    assert res[0][2] == np.asarray(mins1).tolist()
    assert res[0][3] == [np.asarray(lb).tolist() for lb in labels1]
    assert res[0][4] == scores1
    print('faces', faces1, 'kept', res[0][5]['clustered'])


def test_rank_frames_one_global_sequence():
    """rank_frames hands each rank its det-batches of one global frame sequence: with a cycled
    pool the rank's first frame is pool frame (rank's global offset) mod pool; with pool 0 the
    rank's frames are exactly the global sequence's frames [lo, hi) (content depends only on the
    frame index)."""
    import types
    import bench
    from videotofaces import synth
    from videotofaces.parallel import shard_batches
    a = bench.parse(['--det-batch', '4', '--pool', '8'])
    a.H, a.W = 24, 32
    ctx = types.SimpleNamespace(world=3, rank=1, device=torch.device('cpu'))
    frames, off, fnp = bench.rank_frames(a, ctx, 5)
    lo, hi = shard_batches(3 * 5 * 4, 4, 1, 3)
    assert (lo, hi) == (20, 40) and off == lo % 8 and frames.shape[0] == 8 and fnp.shape[0] == 8
    a.pool = 0
    frames, off, fnp = bench.rank_frames(a, ctx, 5)
    ref = synth.make_frames_device(0, 60, 24, 32, seed=1000, style='blobs')
    assert off == 0 and torch.equal(frames, ref[20:40])

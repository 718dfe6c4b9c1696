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

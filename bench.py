"""Benchmark: faces/sec end-to-end (detect + encode) on synthetic frames, 1..8 GPUs of one node.

Workloads (BASELINE.json configs; --config picks the preset, single flags override it):
  c2 (default)  MTCNN (min_face_size=5, RealMTCNN default) + FaceNet bf16, det-batch 16,
                enc-batch 128, 720p frames resident in HBM.  One step = one det-batch per GPU:
                MTCNN (fp32-grade split-fp16 matrix-core convs; pyramid + P/R/O-Net + NMS on device)
                -> box post-processing on device (filter_boxes / adjust_boxes, detection.py:174-262)
                -> crop + INTER_LINEAR resize + FaceNet on device, fed in batches of exactly
                enc-batch (encode_faces, grouping.py:29-40).
  c3            YOLOv3 (fp32, letterbox + Darknet53 + decode + NMS on device) + FaceNet, det-batch 32.
  c4            ViT-L/16 encoder only, enc-batch 128 over pre-cropped 224x224 faces in HBM; one step
                = one enc-batch per GPU.
  c5            YOLOv3 + ViT-L/16 on 1080p frames; after the timed detect+encode region, the
                gathered embeddings go through the cosine dedupe and the K-means k=2..16 sweep
                sharded by k across ranks (timed separately: `grouping`).
The timed region ends with the RCCL all-gather-v of every rank's embeddings (the exchange step
before grouping).  value = faces encoded by all ranks / max-over-ranks wall time.  Without
--steps the detector configs time BASELINE's 10k frames per GPU (625 det-batches of 16): the
per-lane encoder flush at the end of a run (a partial enc-batch per lane) is then amortised as in
a real video, instead of weighing on a 10-20 step sample.

  python bench.py [--gpus N --steps K --warmup W] [--config c2|c3|c4|c5]
With --gpus N > 1 and no torchrun environment the script starts
`torch.distributed.run --nproc-per-node N` itself (before touching a GPU) and exits with its code;
under torchrun WORLD_SIZE must equal --gpus.
"""
import argparse
import json
import os
import socket
import subprocess
import sys
import threading
import time

# Four det-batch lanes (streams) per GPU, each on its own hardware queue: HIP maps a process's
# streams onto GPU_MAX_HW_QUEUES queues (4 on the GPU boxes' environment), so the fourth lane would
# share one.  Set before anything initialises HIP (--hw-queues, default 8; 0 keeps the
# environment's value).  (c2, one box, default run: 3 lanes 9,778 / 9,804 faces/s, 4 lanes on 4
# queues ~9,440, on 8 queues 10,109 / 10,137; profiles/r05ln2_lanes_ab.txt)
def _hw_queues(argv):
    for i, t in enumerate(argv):
        if t == '--hw-queues' and i + 1 < len(argv):
            return int(argv[i + 1])
        if t.startswith('--hw-queues='):
            return int(t.split('=', 1)[1])
    return 8


if _hw_queues(sys.argv[1:]) > 0:
    os.environ['GPU_MAX_HW_QUEUES'] = str(_hw_queues(sys.argv[1:]))

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, 'video-to-faces_amd')):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FP32_PEAK_TFLOPS = 157.3  # MI355X dense fp32 (f32 MFMA), MI355X_MICROARCH.md
BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (no sparsity), MI355X_MICROARCH.md
# split-fp16 operands (x0 w0 + 2^-11 (x0 w1 + x1 w0)): three fp16 products per fp32-grade product
F16X_PEAK_TFLOPS = round(BF16_PEAK_TFLOPS / 3, 1)
# bf16x3 operands (three bf16 terms each): six bf16 products per fp32-grade product
X3_PEAK_TFLOPS = round(BF16_PEAK_TFLOPS / 6, 1)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
VIT_GFLOP = {'vit_b': 11.27, 'vit_l': 39.78}  # per face at 128x128
ENC_NAMES = {'facenet': 'FaceNet', 'vit_b': 'ViT-B/16', 'vit_l': 'ViT-L/16'}
CONFIGS = {
    'c2': dict(det_model='mtcnn', enc_model='facenet', enc_precision='bf16', frame='720p', det_batch=16, pool=0),
    'c3': dict(det_model='yolo', det_precision='x3', enc_model='facenet', enc_precision='bf16', frame='720p',
               det_batch=32, pool=0),
    'c4': dict(det_model='none', enc_model='vit_l', enc_precision='f16x', frame='224'),
    'c5': dict(det_model='yolo', det_precision='x3', enc_model='vit_l', enc_precision='f16x', frame='1080p',
               det_batch=32, grouping=True, pool=0),
}


def parse(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=None,
                    help='timed steps (det-batches or enc-batches); default: the BASELINE frame count '
                         '(--sustain-frames, 10k frames) for detector configs, 20 enc-batches otherwise')
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--config', default='c2', choices=sorted(CONFIGS))
    ap.add_argument('--det-model', choices=['mtcnn', 'yolo', 'none'])
    ap.add_argument('--det-precision', default=None, choices=['fp32', 'x3', 'bf16'],
                    help='YOLO conv precision (default: the config\'s; x3 = fp32-grade bf16x3 products)')
    ap.add_argument('--det-batch', type=int)
    ap.add_argument('--enc-model', choices=['facenet', 'vit_b', 'vit_l'])
    ap.add_argument('--enc-batch', type=int, default=128)
    ap.add_argument('--enc-precision', choices=['bf16', 'fp32', 'f16x'],
                    help='FaceNet: bf16 | fp32; ViT: f16x (guarded split-fp16) | fp32')
    ap.add_argument('--frame', choices=['720p', '1080p', '224'])
    ap.add_argument('--min-face-size', type=float, default=5.0)
    ap.add_argument('--pool', type=int, default=None,
                    help='distinct synthetic frames of the global frame sequence, cycled; 0 (the detector '
                         'configs\' default) = every frame of the timed region distinct, generated on the device')
    ap.add_argument('--touch', type=int, default=1,
                    help='1: read one byte of every 4 KB page of the frames before the timed region')
    ap.add_argument('--lanes', type=int, default=4, help='concurrent det-batch pipelines (threads + HIP streams) per GPU')
    ap.add_argument('--hw-queues', type=int, default=8,
                    help='GPU_MAX_HW_QUEUES for this process (set before HIP starts; 0 = keep the environment)')
    ap.add_argument('--sustain-frames', type=int, default=10000,
                    help='frames of the sustained leg (BASELINE config 2: 10k frames), 0 = skip')
    ap.add_argument('--cpu-frames', type=int, default=None,
                    help='frames per repeat of the CPU-baseline sample (default: BASELINE config 1\'s 64 for '
                         'MTCNN, 16 for YOLO; warm-up 1 frame, min of --cpu-repeats)')
    ap.add_argument('--cpu-repeats', type=int, default=3)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-extras', action='store_true', help='skip the solo / sustained / host-frame / drift legs')
    # box post-processing (detection.py:174-262): the reference's defaults (main.py:18)
    ap.add_argument('--det-min-score', type=float, default=0.4)
    ap.add_argument('--det-min-size', type=int, default=50)
    ap.add_argument('--det-min-border', type=int, default=5)
    a = ap.parse_args(argv)
    preset = CONFIGS[a.config]
    for k in ('det_model', 'det_precision', 'enc_model', 'enc_precision', 'frame', 'det_batch'):
        if getattr(a, k) is None:
            setattr(a, k, preset.get(k))
    if a.det_precision is None:
        a.det_precision = 'fp32'
    a.grouping = preset.get('grouping', False)
    if a.pool is None:
        a.pool = preset.get('pool', 32)
    if a.enc_model == 'facenet' and a.enc_precision == 'f16x':
        a.enc_precision = 'bf16'
    if a.enc_model != 'facenet' and a.enc_precision == 'bf16':
        a.enc_precision = 'f16x'
    yolo = a.det_model == 'yolo'
    if a.det_batch is None:
        a.det_batch = 32 if yolo else 16
    if a.steps is None:
        a.steps = max(1, -(-a.sustain_frames // a.det_batch)) if a.det_model != 'none' and a.sustain_frames > 0 else 20
    if a.cpu_frames is None:
        a.cpu_frames = 16 if yolo else 64
    a.H, a.W = {'720p': (720, 1280), '1080p': (1080, 1920), '224': (224, 224)}[a.frame]
    return a


# ------------------------------------------------------------------ launch
def spawn_command(args_gpus, argv, port):
    """torchrun command line that re-runs this script with one process per GPU."""
    return [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node', str(args_gpus),
            '--master-addr', '127.0.0.1', '--master-port', str(port), os.path.abspath(__file__)] + list(argv)


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def maybe_spawn(args, argv):
    """Called before anything touches a GPU.  Returns an exit code when this process only
    launches (or refuses), None when it should run the benchmark itself."""
    world = os.environ.get('WORLD_SIZE')
    if world is None:
        if args.gpus > 1:
            return subprocess.call(spawn_command(args.gpus, argv, _free_port()))
        return None
    if int(world) != args.gpus:
        print('bench.py: --gpus %d but WORLD_SIZE=%s; launch one process per GPU with '
              'torch.distributed.run --nproc-per-node %d' % (args.gpus, world, args.gpus), file=sys.stderr)
        return 2
    return None


class Ctx:
    """Rank context: process group over RCCL (GPU) or gloo (CPU tests)."""

    def __init__(self, backend='nccl', device=None):
        self.world = int(os.environ.get('WORLD_SIZE', '1'))
        self.rank = int(os.environ.get('RANK', '0'))
        self.local = int(os.environ.get('LOCAL_RANK', '0'))
        self.device = device if device is not None else torch.device('cuda', self.local)
        self.gpu = self.device.type == 'cuda'
        if self.gpu:
            torch.cuda.set_device(self.device)
        if self.world > 1 and not dist.is_initialized():
            if backend == 'nccl':
                dist.init_process_group('nccl', device_id=self.device)
            else:
                dist.init_process_group(backend)

    def sync(self):
        if self.gpu:
            torch.cuda.synchronize(self.device)

    def barrier(self):
        if self.world > 1:
            dist.barrier()

    def reduce(self, values, op):
        t = torch.tensor(values, dtype=torch.float64, device=self.device)
        if self.world > 1:
            dist.all_reduce(t, op=op)
        return [float(v) for v in t.tolist()]

    def gather_rows(self, local):
        if self.world == 1:
            return local
        from videotofaces.parallel import all_gather_rows
        return all_gather_rows(local)

    def close(self):
        if self.world > 1 and dist.is_initialized():
            dist.barrier()
            dist.destroy_process_group()


def measure(pipe, steps, warmup, ctx):
    """Warm-up steps untimed, then exactly `steps` steps bracketed by barrier + device sync on
    both sides, ending with the rank-ordered all-gather of the embeddings.  Returns
    (faces on all ranks, max-over-ranks seconds, gathered embeddings [N,D], per-step faces)."""
    pipe.run(0, warmup)
    ctx.sync()
    ctx.barrier()
    ctx.sync()
    t0 = time.perf_counter()
    stats, parts = pipe.run(warmup, steps)
    local = torch.cat(parts) if parts else torch.zeros((0, pipe.D), device=ctx.device)
    gathered = ctx.gather_rows(local)
    ctx.sync()
    ctx.barrier()
    ctx.sync()
    elapsed = time.perf_counter() - t0
    faces, = ctx.reduce([sum(stats)], dist.ReduceOp.SUM)
    el, = ctx.reduce([elapsed], dist.ReduceOp.MAX)
    return faces, el, gathered, stats


# ------------------------------------------------------------------ GPU pipelines
def _box_params(args):
    from videotofaces import _native as nat
    return nat.BoxParams.make(args.det_min_score, args.det_min_size, args.det_min_border, (1.5, 1.5, 2.2, 1.2), True)


def _make_encoder(args, dev):
    from videotofaces import synth
    if args.enc_model == 'facenet':
        from videotofaces.encoders.facenet import InceptionResnetV1
        return InceptionResnetV1(dev, precision='bf16' if args.enc_precision == 'bf16' else 'fp32')
    from videotofaces.encoders.vit import ViT
    return ViT(dev, synth.make_params(args.enc_model), isL=args.enc_model == 'vit_l',
               precision='fp32' if args.enc_precision == 'fp32' else 'f16x')


def _make_detector(args, dev, fp32=False):
    if args.det_model == 'yolo':
        from videotofaces.detectors.yolo import YOLOv3
        return YOLOv3(dev, precision='fp32' if fp32 else args.det_precision)
    from videotofaces.detectors.mtcnn import MTCNN
    if not fp32:
        return MTCNN(dev)
    old = os.environ.get('VTF_MTCNN_FP32')
    os.environ['VTF_MTCNN_FP32'] = '1'  # read once when the handle is built: all-fp32 MFMA paths
    try:
        return MTCNN(dev)
    finally:
        if old is None:
            del os.environ['VTF_MTCNN_FP32']
        else:
            os.environ['VTF_MTCNN_FP32'] = old


def rank_frames(args, ctx, n_steps, seed=1000):
    """This rank's part of ONE global synthetic frame sequence: the run's world * n_steps
    det-batches split by parallel.shard_batches (whole det-batches, rank order = frame order).
    Returns (frames on the device, offset of the rank's first frame in them, host copy of the
    first max(32, cpu_frames) frames for the CPU-baseline / host-frame / drift legs).
      pool > 0: the sequence cycles `pool` frames (synth.make_frames, seeded; frame g is pool
                frame g % pool), kept on the device once;
      pool = 0: every frame distinct (synth.make_frames_device: frame g's content depends only on
                (seed, g)), the rank's shard generated on the device."""
    from videotofaces import synth
    from videotofaces.parallel import shard_batches
    B = args.det_batch
    lo, hi = shard_batches(ctx.world * n_steps * B, B, ctx.rank, ctx.world)
    if args.pool > 0:
        pool_n = max(B, args.pool // B * B)
        frames_np = synth.make_frames(pool_n, args.H, args.W, seed=seed)
        return torch.from_numpy(frames_np).to(ctx.device), lo % pool_n, frames_np
    # (configs 2 / 3: make_frames' content, on which the detector heads were calibrated; config 5:
    #  faces with identity features for the grouping step)
    frames = synth.make_frames_device(lo, hi, args.H, args.W, seed=seed, device=ctx.device,
                                      style='ids' if args.grouping else 'blobs')
    n_host = max(B, -(-max(32, args.cpu_frames) // B) * B)
    return frames, 0, frames[:n_host].cpu().numpy()


class DetEncPipeline:
    """L lanes of (detector, encoder, HIP stream) on alternate det-batches from host threads (the
    ctypes calls release the GIL): one lane's host syncs and small stage-2/3 kernels overlap
    another lane's pyramid kernel.  Batches stay whole and independent, so per-batch results are
    exactly the single-lane results.  Detector rows never leave HBM: detect_crops returns device
    crop rectangles that the lane's encoder consumes in batches of exactly enc_batch.
    Step i reads frames [offset + i * B, + B) (modulo the frames held) of `frames`, the rank's
    shard of the global sequence (rank_frames).  `make_det` / `make_enc` build one lane's
    detector / encoder (default: the HIP models; tests pass CPU stand-ins)."""

    def __init__(self, args, dev, frames, offset, frames_np, make_det=None, make_enc=None):
        self.args, self.dev = args, dev
        self.B = args.det_batch
        self.frames_np = frames_np
        self.frames = frames
        self.pool_n = frames.shape[0]
        self.offset = offset
        self.L = max(1, args.lanes)
        self.make_det = make_det or (lambda: _make_detector(args, dev))
        self.make_enc = make_enc or (lambda: _make_encoder(args, dev))
        self.dets = [self.make_det() for _ in range(self.L)]
        self.encs = [self.make_enc() for _ in range(self.L)]
        self.D = 512 if args.enc_model == 'facenet' else self.encs[0].dim
        self.gpu = dev.type == 'cuda'
        self.streams = [torch.cuda.Stream(dev) if self.gpu else None for _ in range(self.L)]
        self.bp = _box_params(args) if self.gpu else None
        self.host = None  # host-frame leg: (pinned frames, device ring per lane, slots per lane)
        # lane start-up stagger: lane l starts its first det-batch l x stagger_s after lane 0, so the
        # lanes' pyramid kernels and host syncs are out of step from the first det-batch on, as they
        # are in steady state (all four starting together ran the first det-batches' latency-bound
        # stages 2-3 at the same time: 20-det-batch windows 8.5k -> 9.3k faces/s with 2 ms,
        # 625-det-batch runs unchanged, profiles/r06_lane_stagger_ab.txt; YOLO's 20 ms det-batches
        # of 32: 10 ms, c3 2,468 -> 2,548); env VTF_LANE_STAGGER_MS
        default_ms = {'mtcnn': '2', 'yolo': '10'}.get(args.det_model, '0')
        self.stagger_s = max(0.0, float(os.environ.get('VTF_LANE_STAGGER_MS', default_ms))) / 1e3
        self.minsize = args.min_face_size

    def _stream(self, lane):
        import contextlib
        return torch.cuda.stream(self.streams[lane]) if self.gpu else contextlib.nullcontext()

    def detect_step(self, lane, i, det=None):
        det = det or self.dets[lane]
        if self.host is None:
            j = (self.offset + i * self.B) % self.pool_n
            src, off = self.frames[j:j + self.B], j
        else:  # frames from pinned host memory: async H2D on the lane stream into a ring slot
            pinned, ring, R = self.host[:3]
            j = (i * self.B) % pinned.shape[0]
            slot = lane * R + (i // self.L) % R
            off = slot * self.B
            if len(self.host) == 3:
                ring[off:off + self.B].copy_(pinned[j:j + self.B], non_blocking=True)
            else:  # 4:2:0 planes (the .y4m read path): H2D of 1.5 B/px, then k_yuv_to_bgr into the slot
                from videotofaces import _native as nat
                yring = self.host[3]
                yring[off:off + self.B].copy_(pinned[j:j + self.B], non_blocking=True)
                dst = ring[off:off + self.B]
                nat.check(nat.lib().vtf_yuv_to_bgr(nat.ptr(yring[off:off + self.B]), self.B, dst.shape[1], dst.shape[2],
                                                   420, 0, yring.stride(0), nat.ptr(dst), dst.stride(0), dst.stride(1),
                                                   nat.stream_ptr(self.dev)))
            src = ring[off:off + self.B]
        if self.args.det_model == 'yolo':
            crops, _ = det.detect_crops(src, self.bp, off)
        else:
            crops, _ = det.detect_crops(src, self.minsize, self.bp, off)
        return crops

    def run(self, first, n):
        """steps first..first+n-1, step i on lane i % L -> (faces per step, embeddings per step)."""
        stats = [0] * n
        lane_embs = [[] for _ in range(self.L)]
        errs = []
        eb = self.args.enc_batch
        frames_of = (lambda: self.host[1]) if self.host is not None else (lambda: self.frames)

        stagger_s = self.stagger_s

        def lane_fn(lane):
            try:
                enc = self.encs[lane]
                if stagger_s > 0 and lane > 0:
                    time.sleep(lane * stagger_s)  # (inside the timed region: the start-up policy's cost counts)
                with self._stream(lane):
                    pend, npend, slots = [], 0, []
                    for k in range(lane, n, self.L):
                        if self.host is not None and npend:
                            # the ring slot this step overwrites still holds pending faces: flush
                            R = self.host[2]
                            slot = lane * R + ((first + k) // self.L) % R
                            if slot in slots:
                                lane_embs[lane].append(enc.encode_crops(frames_of(), torch.cat(pend)))
                                pend, npend, slots = [], 0, []
                        crops = self.detect_step(lane, first + k)
                        stats[k] = int(crops.shape[0])
                        if stats[k]:
                            pend.append(crops)
                            npend += stats[k]
                            if self.host is not None:
                                slots.append(lane * self.host[2] + ((first + k) // self.L) % self.host[2])
                        while npend >= eb:
                            allc = torch.cat(pend)
                            lane_embs[lane].append(enc.encode_crops(frames_of(), allc[:eb]))
                            pend = [allc[eb:]] if allc.shape[0] > eb else []
                            npend -= eb
                            if not npend:
                                slots = []
                    if npend:
                        lane_embs[lane].append(enc.encode_crops(frames_of(), torch.cat(pend)))
            except BaseException as e:  # surfaced after join
                errs.append(e)
        ths = [threading.Thread(target=lane_fn, args=(lane,)) for lane in range(self.L)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        if errs:
            raise errs[0]
        for s in self.streams:
            if s is not None:
                s.synchronize()
        # lane streams -> global (step, face) order
        parts, offs = [], [0] * self.L
        flat = [torch.cat(e) if e else torch.zeros((0, self.D), device=self.dev) for e in lane_embs]
        for k in range(n):
            lane, nf = k % self.L, stats[k]
            parts.append(flat[lane][offs[lane]:offs[lane] + nf])
            offs[lane] += nf
        return stats, parts

    # ---- extras
    def solo(self, steps=4):
        """The detector's dominant kernel with the chip to itself: one lane, `steps` det-batches,
        HIP events on the lane stream (vtf_*_profile)."""
        d = self.dets[0]
        d.profile(True)
        stats = []
        with self._stream(0):
            for i in range(steps):
                self.detect_step(0, i)
                stats.append(getattr(d, 'last_stats', None))
        self.streams[0].synchronize()
        self.solo_stats = [st for st in stats if st is not None]
        return d.profile(False)

    def host_frames(self, ring_slots=4, yuv=False):
        """Switch to frames in pinned host memory (None restores HBM-resident frames); yuv=True:
        the frames as 4:2:0 planes (synth.bgr_to_yuv420), converted on the device per det-batch."""
        if ring_slots is None:
            self.host = None
            return
        ring = torch.empty((self.L * ring_slots * self.B,) + tuple(self.frames_np.shape[1:]), dtype=torch.uint8,
                           device=self.dev)
        if not yuv:
            self.host = (torch.from_numpy(self.frames_np).pin_memory(), ring, ring_slots)
            return
        from videotofaces import synth
        planes = torch.from_numpy(synth.bgr_to_yuv420(self.frames_np)).pin_memory()
        yring = torch.empty((ring.shape[0], planes.shape[1]), dtype=torch.uint8, device=self.dev)
        self.host = (planes, ring, ring_slots, yring)

    def drift(self, steps=2):
        """bf16 / split-fp16 perf modes vs the fp32 parity modes on the same det-batches: detector
        boxes (fp32 MFMA detector) and embeddings (fp32 encoder on the same crops)."""
        det32 = _make_detector(self.args, self.dev, fp32=True)
        a = dict(vars(self.args))
        a['enc_precision'] = 'fp32'
        enc32 = _make_encoder(argparse.Namespace(**a), self.dev)
        ious, n_match, n_a, n_b, cos = [], 0, 0, 0, []
        for i in range(steps):
            ca = self.detect_step(0, i).cpu().numpy()
            cb = self.detect_step(0, i, det32).cpu().numpy()
            n_a += len(ca)
            n_b += len(cb)
            for f in np.unique(np.concatenate([ca[:, 0], cb[:, 0]])):
                ra, rb = ca[ca[:, 0] == f, 1:], cb[cb[:, 0] == f, 1:]
                for r in ra:
                    if len(rb):
                        ix = np.clip(np.minimum(r[2], rb[:, 2]) - np.maximum(r[0], rb[:, 0]), 0, None)
                        iy = np.clip(np.minimum(r[3], rb[:, 3]) - np.maximum(r[1], rb[:, 1]), 0, None)
                        inter = ix * iy
                        uni = (r[2] - r[0]) * (r[3] - r[1]) + (rb[:, 2] - rb[:, 0]) * (rb[:, 3] - rb[:, 1]) - inter
                        best = float((inter / np.maximum(uni, 1)).max())
                        ious.append(best)
                        n_match += best == 1.0
            if len(ca):
                dc = torch.from_numpy(ca).to(self.dev)
                e16 = self.encs[0].encode_crops(self.frames, dc)
                e32 = enc32.encode_crops(self.frames, dc)
                cos.append(torch.nn.functional.cosine_similarity(e16, e32, dim=1).cpu().numpy())
        cos = np.concatenate(cos) if cos else np.zeros(0)
        return {'det_batches': steps, 'faces_perf_mode': n_a, 'faces_fp32_mode': n_b,
                'crop_rect_identical_frac': round(n_match / max(1, n_a), 4),
                'crop_iou_mean': round(float(np.mean(ious)), 6) if ious else None,
                'crop_iou_min': round(float(np.min(ious)), 6) if ious else None,
                'embedding_cos_mean': round(float(cos.mean()), 6) if len(cos) else None,
                'embedding_cos_min': round(float(cos.min()), 6) if len(cos) else None,
                'enc_modes': '%s vs fp32' % self.args.enc_precision,
                'det_modes': ('split-fp16 vs fp32 MFMA' if self.args.det_model == 'mtcnn'
                              else '%s vs fp32' % self.args.det_precision)}


class EncodePipeline:
    """BASELINE config 4: pre-cropped 224x224 faces resident in HBM, one enc-batch per step
    (blob 224 -> 128 + ViT forward, one stream)."""

    def __init__(self, args, dev, rank):
        from videotofaces import synth
        self.args, self.dev, self.B = args, dev, args.enc_batch
        # every crop of the warm-up + timed steps distinct (2,944 crops = 443 MB at the defaults:
        # larger than the 256 MB Infinity Cache, so the reads come from HBM)
        self.pool_n = max(self.B, (max(args.warmup, 1) + args.steps) * self.B)
        self.crops_u8 = torch.from_numpy(synth.make_crops(self.pool_n, 224, seed=1 + rank)).to(dev)
        self.boxes = torch.tensor([[i, 0, 0, 224, 224] for i in range(self.pool_n)], dtype=torch.int32, device=dev)
        self.enc = _make_encoder(args, dev)
        self.D = 512 if args.enc_model == 'facenet' else self.enc.dim

    def run(self, first, n):
        stats, parts = [], []
        for i in range(first, first + n):
            j = (i * self.B) % self.pool_n
            parts.append(self.enc.encode_crops(self.crops_u8, self.boxes[j:j + self.B]))
            stats.append(self.B)
        return stats, parts


# ------------------------------------------------------------------ CPU baseline (oracle)
def _cores():
    n = len(os.sched_getaffinity(0))
    env = os.environ.get('OMP_NUM_THREADS')
    return min(n, int(env)) if env and env.isdigit() else n


def cpu_baseline(args, frames_np):
    """The oracle (CPU restatement of the reference path: torch-CPU nets, C NMS, numpy box logic)
    on a bounded sample of the same workload, rank 0 only, with BASELINE.md §2's protocol: one
    untimed warm-up, then the minimum over `cpu_repeats` timed repeats of the sample.  Detection
    runs at det-batch 1, the BASELINE config-1 shape (the reference CPU path); the sample is the
    first `cpu_frames` frames of config 1's 64 (a stated reduction, to keep the default run within
    minutes)."""
    from oracle.boxes import rows_to_crops
    from oracle.facenet import inception_resnet_v1, resize_linear_u8
    from oracle.vit import vit
    from videotofaces import synth
    cores = _cores()
    torch.set_num_threads(cores)
    pf = synth.make_params(args.enc_model)
    vit_dims = {'vit_b': (768, 12), 'vit_l': (1024, 24)}.get(args.enc_model)

    def encode(imgs):
        blobs = []
        for im in imgs:
            if vit_dims:  # blobFromImages(1/127.5, 128x128, 127.5, swapRB) (vit.py:141)
                r = resize_linear_u8(im, 128)[:, :, ::-1].transpose(2, 0, 1)
                blobs.append((torch.from_numpy(np.ascontiguousarray(r)).float() - 127.5) * (1 / 127.5))
            else:  # blobFromImages(1/128, 160x160, 127.5, swapRB) (facenet.py:179)
                r = resize_linear_u8(im, 160)[:, :, ::-1].transpose(2, 0, 1)
                blobs.append((torch.from_numpy(np.ascontiguousarray(r)).float() - 127.5) * (1 / 128))
        for i in range(0, len(blobs), args.enc_batch):
            x = torch.stack(blobs[i:i + args.enc_batch])
            vit(pf, x, *vit_dims) if vit_dims else inception_resnet_v1(pf, x)

    def best_of(run):
        run(1)  # warm-up (untimed)
        ts = []
        for _ in range(max(1, args.cpu_repeats)):
            t0 = time.perf_counter()
            faces = run(None)
            ts.append(time.perf_counter() - t0)
        return faces, min(ts), ts

    proto = 'warm-up 1, min of %d repeats' % max(1, args.cpu_repeats)
    if args.det_model == 'none':
        n = 16
        crops = list(synth.make_crops(n, 224, seed=2))
        faces, dt, ts = best_of(lambda w: (encode(crops[:w or n]), w or n)[1])
        return {'value': round(faces / dt, 3), 'unit': 'faces/s', 'cores': cores, 'kind': 'port',
                'repeats_s': [round(t, 2) for t in ts], 'protocol': proto,
                'sample': '%d synthetic 224x224 crops, oracle %s fp32 on CPU, %s, best %.1f s'
                          % (n, ENC_NAMES[args.enc_model], proto, dt)}
    from oracle import mtcnn as om
    from oracle import yolo as oy
    pm = synth.make_params(args.det_model)
    n = min(args.cpu_frames, frames_np.shape[0])

    def run(w):
        imgs = []
        for f in range(w or n):  # det-batch 1 (config 1)
            if f % 8 == 0:  # progress on stderr (a minutes-long leg: keep watchdogs informed)
                print('cpu_baseline: frame %d of %d' % (f, w or n), file=sys.stderr, flush=True)
            fr = frames_np[f:f + 1]
            if args.det_model == 'yolo':
                b, s, _ = oy.forward(pm, list(fr))
                res = [np.concatenate([b[0], s[0][:, None]], 1)]
            else:
                res = om.forward(pm, list(fr), minsize=args.min_face_size)
            crops, _ = rows_to_crops(res, (args.H, args.W), args.det_min_score, args.det_min_size,
                                     args.det_min_border, (1.5, 1.5, 2.2, 1.2), True)
            imgs.extend(fr[0, y1:y2, x1:x2] for _, x1, y1, x2, y2 in crops)
        encode(imgs)
        return len(imgs)

    faces, dt, ts = best_of(run)
    det = 'YOLOv3' if args.det_model == 'yolo' else 'MTCNN(min_face_size=%g)' % args.min_face_size
    return {'value': round(faces / dt, 3), 'unit': 'faces/s', 'cores': cores, 'kind': 'port',
            'repeats_s': [round(t, 2) for t in ts], 'protocol': proto,
            'sample': '%d synthetic %s frames at det-batch 1 (%d faces; config 1 is 64 frames), oracle %s + box '
                      'logic + %s fp32 on CPU, %s, best %.1f s'
                      % (n, args.frame, faces, det, ENC_NAMES[args.enc_model], proto, dt)}


# ------------------------------------------------------------------ roofline
def roofline_det(args, pipe, shared, solo):
    """Dominant detector kernel: k_pnet (MTCNN) or the YOLO conv stack.  `avg_launch_ms` is the
    kernel's own duration with the chip to itself (solo leg, one lane; it matches a one-lane
    rocprofv3 trace); the concurrent-lane figure (events spanning co-running kernels of the
    other lanes) is kept under `shared`."""
    yolo = args.det_model == 'yolo'
    s_ms, s_n, s_fl, _ = solo
    c_ms, c_n, c_fl, _ = shared
    s_avg, c_avg = s_ms / max(1, s_n), c_ms / max(1, c_n)
    fl = s_fl / max(1, s_n)
    if yolo:
        peak = {'bf16': BF16_PEAK_TFLOPS, 'x3': X3_PEAK_TFLOPS}.get(args.det_precision, FP32_PEAK_TFLOPS)
        kname = ('k_conv_dma3 (YOLOv3 Darknet53+neck+head, 75 implicit-GEMM launches per det-batch, bf16x3 operands: '
                 'fp32-grade; peak = bf16 dense / 6 products)' if args.det_precision == 'x3' else
                 'k_conv (YOLOv3 Darknet53+neck+head, 75 implicit-GEMM launches per det-batch, %s)' % args.det_precision)
    else:
        peak = F16X_PEAK_TFLOPS
        kname = ('k_pnet (fused pyramid resample + PNet; convs on fp16 matrix cores with split operands, '
                 'fp32-grade; peak = fp16 dense / 3 products; one "launch" = the det-batch\'s exact-levels '
                 'k_pnet<false,true,false> + pre-resampled k_pnet<false,false,true> pair: rocprof lists them as '
                 'two rows; the downsampled levels\' resample runs before, in k_resample_sat_multi)')
    ach = fl / (s_avg / 1e3) / 1e12 if s_avg > 0 else 0.0
    c_ach = (c_fl / max(1, c_n)) / (c_avg / 1e3) / 1e12 if c_avg > 0 else 0.0
    traffic = None
    tf = os.path.join(ROOT, 'profiles', ('yolo' if yolo else 'pnet') + '_traffic.json')
    if os.path.exists(tf) and not (yolo and args.det_precision != 'fp32'):  # measured for the fp32 YOLO / k_pnet
        traffic = json.load(open(tf)).get('hbm_bytes_per_launch')
    r = {'kernel': kname, 'bound': 'mfma', 'achieved': round(ach, 3), 'peak': peak, 'unit': 'TFLOP/s',
         'frac': round(ach / peak, 4), 'traffic': traffic, 'avg_launch_ms': round(s_avg, 4),
         'flops_per_launch': fl, 'launches': s_n, 'timing': 'solo leg: one lane, HIP events on its stream',
         'shared': {'avg_launch_ms': round(c_avg, 4), 'achieved': round(c_ach, 3), 'frac': round(c_ach / peak, 4),
                    'launches': c_n, 'concurrent_lanes': pipe.L}}
    return r, None


# RNet / ONet FLOPs per candidate (2 x MACs of every conv and dense layer, mtcnn.py:41-109):
# RNet 24x24: conv1 22^2*28*27, conv2 9^2*48*252, conv3 3^2*64*192, dense 576*128, heads 128*6;
# ONet 48x48: conv1 46^2*32*27, conv2 21^2*64*288, conv3 8^2*64*576, conv4 3^2*128*256,
# dense 1152*256, heads 256*16
RNET_FLOP = 2 * (22 * 22 * 28 * 27 + 9 * 9 * 48 * 252 + 9 * 64 * 192 + 576 * 128 + 128 * 6)
ONET_FLOP = 2 * (46 * 46 * 32 * 27 + 21 * 21 * 64 * 288 + 64 * 64 * 576 + 9 * 128 * 256 + 1152 * 256 + 256 * 16)


def roofline_e2e(args, faces_per_step, ms_per_step, solo, solo_stats):
    """SURVEY.md §8d's end-to-end bound: faces/s roofline = faces / sum over the stages of
    max(FLOPs / peak, bytes / HBM BW), per GPU and per step (one det-batch, or one enc-batch for
    the encoder-only config).  Stage FLOPs are the algorithmic counts (pyramid+PNet from the
    level plan, RNet / ONet per candidate x the candidates the detector passed in the solo leg,
    the encoder per face); peaks are the ones the stages compute at (split-fp16 / bf16x3 for
    the fp32-grade detector convs, the encoder's mode); bytes are the stage's compulsory input
    (frames, or the uint8 crops).  `frac` = achieved faces/s per GPU / roofline faces/s."""
    stages = []

    def add(name, flops, peak, nbytes):
        t = max(flops / (peak * 1e12), nbytes / (HBM_PEAK_GBS * 1e9))
        stages.append({'stage': name, 'gflop': round(flops / 1e9, 3), 'peak_tflops': peak,
                       'mbytes': round(nbytes / 1e6, 3), 'bound_us': round(t * 1e6, 2)})
    enc_gf = 2.835 if args.enc_model == 'facenet' else VIT_GFLOP[args.enc_model]
    if args.enc_model == 'facenet':
        enc_peak = BF16_PEAK_TFLOPS if args.enc_precision == 'bf16' else FP32_PEAK_TFLOPS
    else:
        enc_peak = FP32_PEAK_TFLOPS if args.enc_precision == 'fp32' else F16X_PEAK_TFLOPS
    side = 160 if args.enc_model == 'facenet' else 128
    if args.det_model != 'none' and solo is not None:
        s_ms, s_n, s_fl, s_frames = solo
        fl = s_fl / max(1.0, s_frames / args.det_batch)  # per det-batch (YOLO counts a launch per conv)
        frame_bytes = args.det_batch * args.H * args.W * 3
        if args.det_model == 'yolo':
            peak = {'bf16': BF16_PEAK_TFLOPS, 'x3': X3_PEAK_TFLOPS}.get(args.det_precision, FP32_PEAK_TFLOPS)
            add('YOLOv3 (letterbox + Darknet53 + neck + heads)', fl, peak, frame_bytes)
        else:
            add('pyramid + PNet', fl, F16X_PEAK_TFLOPS, frame_bytes)
            st = np.array(solo_stats, dtype=np.float64) if solo_stats else None
            n2 = float(st[:, 3].mean()) if st is not None else 0.0
            n3 = float(st[:, 5].mean()) if st is not None else 0.0
            add('RNet (%.0f candidates)' % n2, n2 * RNET_FLOP, F16X_PEAK_TFLOPS, n2 * 24 * 24 * 3 * 4)
            add('ONet (%.0f candidates)' % n3, n3 * ONET_FLOP, F16X_PEAK_TFLOPS, n3 * 48 * 48 * 3 * 4)
    add('%s (%.1f faces)' % (ENC_NAMES[args.enc_model], faces_per_step), faces_per_step * enc_gf * 1e9, enc_peak,
        faces_per_step * side * side * 3)
    bound_ms = sum(x['bound_us'] for x in stages) / 1e3
    roof = faces_per_step / (bound_ms / 1e3) if bound_ms > 0 else None
    ach = faces_per_step / (ms_per_step / 1e3) if ms_per_step > 0 else 0.0
    return {'faces_per_s_per_gpu': round(ach, 2), 'roofline_faces_per_s_per_gpu': round(roof, 2) if roof else None,
            'frac': round(ach / roof, 4) if roof else None, 'bound_ms_per_step': round(bound_ms, 4),
            'ms_per_step': round(ms_per_step, 4), 'stages': stages,
            'note': 'SURVEY.md 8d: faces / sum_stages max(FLOPs/peak, bytes/BW); per GPU, per det-batch'}


def roofline_enc(args, ms_per_step):
    if args.enc_model == 'facenet':
        peak = BF16_PEAK_TFLOPS if args.enc_precision == 'bf16' else FP32_PEAK_TFLOPS
        ach = 2.835 * args.enc_batch / ms_per_step  # 2.835 GFLOP per face
        return {'kernel': 'whole FaceNet encoder step (blob + k_conv %s + pools + head)' % args.enc_precision,
                'bound': 'mfma', 'achieved': round(ach, 3), 'peak': peak, 'unit': 'TFLOP/s',
                'frac': round(ach / peak, 4), 'traffic': None, 'avg_launch_ms': round(ms_per_step, 4),
                'flops_per_launch': 2.835e9 * args.enc_batch, 'timing': 'one enc-batch per step'}
    peak = FP32_PEAK_TFLOPS if args.enc_precision == 'fp32' else F16X_PEAK_TFLOPS
    ach = VIT_GFLOP[args.enc_model] * args.enc_batch / ms_per_step
    return {'kernel': 'whole ViT encoder step (blob + k_conv split-fp16 GEMMs + attention + LayerNorm)',
            'bound': 'mfma', 'achieved': round(ach, 3), 'peak': peak, 'unit': 'TFLOP/s', 'frac': round(ach / peak, 4),
            'traffic': None, 'avg_launch_ms': round(ms_per_step, 4),
            'flops_per_launch': VIT_GFLOP[args.enc_model] * 1e9 * args.enc_batch,
            'timing': 'one enc-batch per step, wall clock of the timed region'}


# ------------------------------------------------------------------ main
def grouping_leg(X, ctx, dev, rows_fn=None, grouper=None):
    """main.py:72-77 on the gathered embeddings X (every rank holds them): the cosine dedupe
    (dupes.py:60-65) row-sharded across the ranks, then KMeans + silhouette / CH / DB for
    k = 2..16 on the kept rows (grouping.py:97-107), sharded by k and by silhouette rows.
    rows_fn / grouper replace the device kernels (CPU tests).  Returns (record, mins, labels,
    scores); times are max over ranks."""
    from videotofaces import dupes
    from videotofaces.grouping import cluster_sweep
    X = X.contiguous()
    if ctx.world > 1:  # once, outside the timed region: every rank holds the same gathered X (then
        # the kept rows are replicated too: mins are all-gathered), so the timed calls skip the digest
        from videotofaces.parallel import check_replicated
        check_replicated(X.cpu().numpy(), 'grouping_leg')
    ctx.sync()
    ctx.barrier()
    t0 = time.perf_counter()
    if rows_fn is None:
        mins, _ = dupes.cosine_dedupe_device(X, sharded=True, replicated=True)
    else:
        Xh = X.cpu().numpy()
        mins, _ = dupes.cosine_dedupe_sharded(Xh, rows_fn) if ctx.world > 1 else rows_fn(0, Xh.shape[0])
    ctx.sync()
    t_dd = time.perf_counter() - t0
    Xk = X.cpu().numpy()[~(mins <= 0.25)]
    ks = [k for k in range(2, 17) if k <= Xk.shape[0]]
    t1 = time.perf_counter()
    labels, scores = cluster_sweep(Xk, ks, 0, grouper=grouper, device=dev, sharded=True, replicated=True)
    ctx.sync()
    t_sw = time.perf_counter() - t1
    ctx.barrier()
    tg, t_dd, t_sw = ctx.reduce([time.perf_counter() - t0, t_dd, t_sw], dist.ReduceOp.MAX)
    best = max(scores, key=lambda s: s[1])[0] if scores else None
    rec = {'faces': int(X.shape[0]), 'dupes_at_0.25': int((mins <= 0.25).sum()), 'clustered': int(Xk.shape[0]),
           'clustered_frac': round(Xk.shape[0] / max(1, X.shape[0]), 4),
           'k': [ks[0], ks[-1]] if ks else [], 'seconds': round(tg, 4), 'dedupe_s': round(t_dd, 4),
           'sweep_s': round(t_sw, 4), 'best_k_silhouette': best,
           'note': 'fused cosine dedupe of the gathered embeddings (rows sharded across ranks), then KMeans + '
                   'silhouette/CH/DB for each k on the kept rows (main.py:72-77), k sharded across ranks '
                   '(max over ranks)'}
    return rec, mins, labels, scores


def run_gpu(args):
    ctx = Ctx('nccl')
    dev = ctx.device
    if args.det_model == 'none':
        pipe = EncodePipeline(args, dev, ctx.rank)
    else:
        warm = max(args.warmup, max(1, args.lanes))
        frames, offset, frames_np = rank_frames(args, ctx, warm + args.steps)
        if args.touch:
            # frames resident in HBM: one byte per 4 KB page read once (the page translations warm,
            # as for a video pipeline's reused frame buffers; 1/4096 of the bytes, far below the
            # 256 MB Infinity Cache's reach over the run's frames), outside the timed region
            frames.view(-1)[::4096].sum()
        pipe = DetEncPipeline(args, dev, frames, offset, frames_np)
    ctx.sync()
    faces, elapsed, gathered, _ = measure(pipe, args.steps, max(args.warmup, getattr(pipe, 'L', 1)), ctx)
    det = args.det_model != 'none'
    shared = None
    if det:
        for d in pipe.dets:
            d.profile(True)
        pipe.run(0, len(pipe.dets))  # one det-batch per lane with timing on (events, concurrent lanes)
        shared = [0, 0, 0, 0]
        for d in pipe.dets:
            shared = [a + b for a, b in zip(shared, d.profile(False))]
    out = {}
    extras = not args.no_extras
    if det and extras:
        solo = pipe.solo(4)
        # sustained leg: BASELINE config 2's 10k frames (per rank) through the same pipeline
        n_sus = max(1, -(-args.sustain_frames // args.det_batch)) if args.sustain_frames > 0 else 0
        if n_sus > args.steps:  # (the default timed region already covers the BASELINE frame count)
            f_sus, t_sus, _, _ = measure(pipe, n_sus, 0, ctx)
            out['sustained'] = {'frames_per_rank': n_sus * args.det_batch, 'steps': n_sus,
                                'value': round(f_sus / t_sus, 2), 'seconds': round(t_sus, 3),
                                'ms_per_step': round(t_sus * 1e3 / n_sus, 3)}
        # PCIe-inclusive variant: frames from pinned host memory, async H2D on each lane's stream
        pipe.host_frames(4)
        f_h, t_h, _, _ = measure(pipe, args.steps, pipe.L, ctx)
        pipe.host_frames(None)
        out['host_frames'] = {'value': round(f_h / t_h, 2), 'ms_per_step': round(t_h * 1e3 / args.steps, 3),
                              'faces_per_frame': round(f_h / max(1, ctx.world * args.steps * args.det_batch), 3),
                              'note': 'frames start in pinned host memory (the host frame pool, cycled: its content '
                                      'differs from the distinct device frames, compare ms_per_step); H2D (%.1f MB '
                                      'per det-batch) inside the timed region' % (args.det_batch * args.H * args.W * 3 / 1e6)}
        # the .y4m frame source's device half: 4:2:0 planes in pinned host memory, H2D of 1.5 B/px
        # and k_yuv_to_bgr per det-batch (videotofaces/video.py; the file gather is host work)
        if args.det_model == 'mtcnn' and args.H % 2 == 0 and args.W % 2 == 0:
            pipe.host_frames(4, yuv=True)
            f_y, t_y, _, _ = measure(pipe, args.steps, pipe.L, ctx)
            pipe.host_frames(None)
            out['host_yuv_frames'] = {
                'value': round(f_y / t_y, 2), 'ms_per_step': round(t_y * 1e3 / args.steps, 3),
                'faces_per_frame': round(f_y / max(1, ctx.world * args.steps * args.det_batch), 3),
                'note': 'frames start as 4:2:0 planes in pinned host memory (the .y4m read path): H2D (%.1f MB per '
                        'det-batch) + k_yuv_to_bgr inside the timed region; the decoded frames differ from the BGR '
                        'originals by the 4:2:0 round trip' % (args.det_batch * args.H * args.W * 1.5 / 1e6)}
        if ctx.rank == 0:
            out['bf16_drift'] = pipe.drift(2)
    elif det:
        solo = pipe.solo(2)
    grouping = None
    if args.grouping:
        grouping = grouping_leg(gathered, ctx, dev)[0]
        # The random-weight encoder maps synthetic faces close together, so at ~10k faces most
        # rows have an earlier neighbour within the 0.25 dedupe threshold.  A second leg grows
        # a long-video set from the gathered rows (synth.video_embeddings: 40 identities + 40 %
        # detector junk + noise, the generator of the 30k scale golden) at N = 30k, where the
        # dedupe keeps a realistic share, and times the same sharded dedupe + k sweep on it.
        from videotofaces import synth
        Xg = gathered.cpu().numpy()
        Xv = synth.video_embeddings(Xg[np.unique(Xg, axis=0, return_index=True)[1]], 30000, seed=5)
        rec = grouping_leg(torch.from_numpy(Xv).to(dev), ctx, dev)[0]
        rec['note'] = ('synth.video_embeddings(gathered rows, 30000, seed=5): ' + rec['note'])
        out['grouping_video'] = rec
    if ctx.rank == 0:
        steps = args.steps
        frames_all = ctx.world * steps * (args.det_batch if det else 0)
        dtype_enc = args.enc_precision if args.enc_precision != 'f16x' else 'fp32 (split-fp16 MFMA)'
        if det:
            roof, _ = roofline_det(args, pipe, shared, solo)
            wl = ('YOLOv3(%s)' % args.det_precision if args.det_model == 'yolo'
                  else 'MTCNN(min_face_size=%g)' % args.min_face_size) + '+' + ENC_NAMES[args.enc_model]
            dtype = '%s det / %s enc' % (args.det_precision if args.det_model == 'yolo' else 'fp32 (split-fp16 MFMA)',
                                         dtype_enc)
            workload = ('%s, det-batch %d, enc-batch %d, %s, frames in HBM, box filter min_score %g min_size %d '
                        'min_border %d, det_scale (1.5,1.5,2.2,1.2), square' % (
                            wl, args.det_batch, args.enc_batch, args.frame, args.det_min_score, args.det_min_size,
                            args.det_min_border))
            metric = 'faces/sec end-to-end (detect+encode) on %dx%d synthetic frames' % (args.W, args.H)
        else:
            roof = roofline_enc(args, elapsed * 1e3 / steps)
            dtype = dtype_enc
            workload = '%s encoder only, enc-batch %d, pre-cropped 224x224 uint8 faces in HBM' % (
                ENC_NAMES[args.enc_model], args.enc_batch)
            metric = 'faces/sec, %s encoder on pre-cropped 224x224 faces' % ENC_NAMES[args.enc_model]
        res = {
            'metric': metric, 'value': round(faces / elapsed, 2), 'unit': 'faces/s', 'n_gpus': ctx.world,
            'steps': steps, 'warmup': args.warmup, 'ms_per_step': round(elapsed * 1e3 / steps, 3),
            'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': dtype,
            'data': 'synthetic (seeded %s frames/crops; hash-seeded synthetic weights, detector heads calibrated '
                    'to a few face-sized detections per frame, encoders calibrated to spread embeddings)' % args.frame,
            'config': {'workload': workload, 'baseline_config': args.config, 'det_batch': args.det_batch if det else None,
                       'enc_batch': args.enc_batch, 'frames_per_step_per_gpu': args.det_batch if det else 0,
                       'lanes': getattr(pipe, 'L', 1), 'hw_queues': os.environ.get('GPU_MAX_HW_QUEUES'),
                       'lane_stagger_ms': round(getattr(pipe, 'stagger_s', 0.0) * 1e3, 3),
                       'parallelism': 'dp%d (frame-sharded, RCCL all-gather of embeddings)' % ctx.world,
                       # the reference writes face crops as JPEG files and re-reads them for the
                       # encoder (detection.py -> encoders); here crops go from HBM frames to the
                       # encoder without that round trip, as without video decode
                       'excluded': 'video decode, JPEG write/read of crops, file moves',
                       'pool': args.pool,
                       'frame_source': ('every frame distinct, generated on the device from (seed, frame index) '
                                        'before the timed region (--pool 0, style %s)' % ('ids' if args.grouping else 'blobs')
                                        if det and args.pool == 0 else
                                        ('a %d-frame pool cycled (--pool %d)' % (args.pool, args.pool) if det else
                                         'pre-cropped faces'))},
            'faces_per_frame': round(faces / max(1, frames_all), 3) if det else None,
            'frames_per_s': round(frames_all / elapsed, 2) if det else None,
            'embeddings_gathered': int(gathered.shape[0]),
            'roofline': roof,
            'roofline_e2e': roofline_e2e(args, faces / max(1, ctx.world * steps), elapsed * 1e3 / steps,
                                         solo if det else None, getattr(pipe, 'solo_stats', None)),
            'cpu_baseline': None,
        }
        res.update(out)
        if grouping:
            res['grouping'] = grouping
        if ctx.world == 1 and not args.no_cpu_baseline:
            res['cpu_baseline'] = cpu_baseline(args, getattr(pipe, 'frames_np', None))
        print(json.dumps(res), flush=True)
    ctx.close()


def main(argv=None):
    argv = sys.argv[1:] if argv is None else argv
    args = parse(argv)
    rc = maybe_spawn(args, argv)
    if rc is not None:
        sys.exit(rc)
    run_gpu(args)


if __name__ == '__main__':
    main()

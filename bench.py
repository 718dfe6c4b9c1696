"""Benchmark: faces/sec end-to-end (detect + encode) on synthetic 1280x720 frames.

Workload (BASELINE.json configs[1]): MTCNN (min_face_size=5, RealMTCNN default) + FaceNet,
det-batch 16, enc-batch 128, frames resident in HBM.  One step = one det-batch per GPU:
  MTCNN detect (fp32-grade: split-fp16 matrix-core convs; pyramid + P/R/O-Net + NMS on device)
  -> reference box post-processing (filter_boxes / adjust_boxes, detection.py:174-262, host)
  -> crop + INTER_LINEAR resize + FaceNet on device (bf16 by default; --enc-precision fp32).
--det-model yolo runs configs[2] instead: YOLOv3 (letterbox + Darknet53 + decode + NMS on
device, fp32 or --det-precision bf16) + FaceNet, det-batch 32.
The timed region ends with the RCCL all-gather-v of every rank's embeddings (the exchange
step before grouping).  value = faces encoded by all ranks / max-over-ranks wall time.

  python bench.py [--gpus N --steps K --warmup W]
  torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU, RCCL)
"""
import argparse
import json
import os
import sys
import threading
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'video-to-faces_amd')]

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

FP32_PEAK_TFLOPS = 157.3  # MI355X dense fp32 (vector = f32 MFMA), MI355X_MICROARCH.md
BF16_PEAK_TFLOPS = 2500.0  # MI355X dense bf16 MFMA (no sparsity), MI355X_MICROARCH.md
# k_pnet's convs run on the fp16 matrix cores with split operands (x0 w0 + 2^-11 (x0 w1 + x1 w0):
# three fp16 products per fp32-grade product), so its fp32-equivalent ceiling is fp16 dense / 3
F16X_PEAK_TFLOPS = round(BF16_PEAK_TFLOPS / 3, 1)
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E (MI355X_MICROARCH.md)
LBL_BYTES_PER_FLOP = 2075e6 / 38.66e9  # PNet layer-by-layer fp32 bytes per FLOP
H, W = 720, 1280  # --frame 1080p: 1080, 1920
ENC_NAMES = {'facenet': 'FaceNet', 'vit_b': 'ViT-B/16', 'vit_l': 'ViT-L/16'}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=3)
    ap.add_argument('--det-model', default='mtcnn', choices=['mtcnn', 'yolo'])
    ap.add_argument('--det-precision', default='fp32', choices=['fp32', 'bf16'], help='YOLO conv precision')
    ap.add_argument('--det-batch', type=int, default=None, help='default 16 (mtcnn) / 32 (yolo)')
    ap.add_argument('--enc-batch', type=int, default=128)
    ap.add_argument('--enc-precision', default='bf16', choices=['bf16', 'fp32'])
    ap.add_argument('--min-face-size', type=float, default=5.0)
    ap.add_argument('--pool', type=int, default=32, help='distinct synthetic frames per rank (cycled)')
    ap.add_argument('--lanes', type=int, default=3, help='concurrent det-batch pipelines (threads + HIP streams) per GPU')
    ap.add_argument('--cpu-frames', type=int, default=None,
                    help='frames in the bounded CPU-baseline sample (default 12 mtcnn / 32 yolo, ~10 s of CPU work)')
    ap.add_argument('--no-cpu-baseline', action='store_true')
    # box post-processing (detection.py:174-262): reference defaults except det_min_size,
    # because synthetic-weight detections are mostly < 50 px and would never reach the encoder
    ap.add_argument('--det-min-score', type=float, default=0.4)
    ap.add_argument('--det-min-size', type=int, default=None, help='default 0 (mtcnn) / 50 (yolo)')
    ap.add_argument('--det-min-border', type=int, default=5)
    ap.add_argument('--enc-model', default='facenet', choices=['facenet', 'vit_b', 'vit_l'],
                    help='vit_*: ViT-B/L-16 encoder (BASELINE config 5 pairs YOLO with ViT-L); '
                         'its GEMMs run split-fp16 unless --enc-precision fp32')
    ap.add_argument('--frame', default='720p', choices=['720p', '1080p'])
    a = ap.parse_args()
    global H, W
    H, W = (1080, 1920) if a.frame == '1080p' else (720, 1280)
    yolo = a.det_model == 'yolo'
    if a.det_batch is None:
        a.det_batch = 32 if yolo else 16
    if a.det_min_size is None:
        a.det_min_size = 50 if yolo else 0
    if a.cpu_frames is None:
        a.cpu_frames = 32 if yolo else 12
    return a


def det_params(args):
    return dict(mscore=args.det_min_score, msize=args.det_min_size, mborder=args.det_min_border,
                scale=(1.5, 1.5, 2.2, 1.2), square=True)


def cpu_baseline(frames, args):
    """The oracle (CPU restatement of the reference path, torch-CPU + C NMS) on a bounded
    sample of the same workload, rank 0 only."""
    from oracle import mtcnn as om
    from oracle import yolo as oy
    from oracle.facenet import inception_resnet_v1, resize_linear_u8
    from oracle.vit import vit
    from videotofaces import synth
    from videotofaces.detection import boxes_to_crops
    cores = len(os.sched_getaffinity(0))
    env = os.environ.get('OMP_NUM_THREADS')
    if env and env.isdigit():
        cores = min(cores, int(env))
    torch.set_num_threads(cores)
    yolo = args.det_model == 'yolo'
    pm, pf = synth.make_params(args.det_model), synth.make_params(args.enc_model)
    vit_dims = {'vit_b': (768, 12), 'vit_l': (1024, 24)}.get(args.enc_model)
    n = min(args.cpu_frames, frames.shape[0])
    sample = frames[:n]
    t0 = time.time()
    if yolo:
        res = oy.forward(pm, list(sample))
    else:
        res = om.forward(pm, list(sample), minsize=args.min_face_size)
    crops = boxes_to_crops(res, (H, W), **det_params(args))
    faces = 0
    for i in range(0, crops.shape[0], args.enc_batch):
        blobs = []
        for f, x1, y1, x2, y2 in crops[i:i + args.enc_batch]:
            if vit_dims:  # blobFromImages(1/127.5, 128x128, 127.5, swapRB) (vit.py:141)
                r = resize_linear_u8(sample[f, y1:y2, x1:x2], 128)[:, :, ::-1].transpose(2, 0, 1)
                blobs.append((torch.from_numpy(np.ascontiguousarray(r)).float() - 127.5) * (1 / 127.5))
            else:
                r = resize_linear_u8(sample[f, y1:y2, x1:x2], 160)[:, :, ::-1].transpose(2, 0, 1)
                blobs.append((torch.from_numpy(np.ascontiguousarray(r)).float() - 127.5) * (1 / 128))
        if vit_dims:
            vit(pf, torch.stack(blobs), *vit_dims)
        else:
            inception_resnet_v1(pf, torch.stack(blobs))
        faces += len(blobs)
    dt = time.time() - t0
    return {'value': round(faces / dt, 3), 'unit': 'faces/s', 'cores': cores, 'kind': 'port',
            'sample': '%d synthetic %s frames (%d faces), oracle %s+%s fp32 on CPU, %.1f s'
                      % (n, args.frame, faces, 'YOLOv3' if yolo else 'MTCNN(min_face_size=%g)' % args.min_face_size,
                         ENC_NAMES[args.enc_model], dt)}


def main():
    args = parse()
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    if world > 1:
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
    dev = torch.device('cuda', local)
    from videotofaces import synth
    from videotofaces.detectors.mtcnn import MTCNN
    from videotofaces.detectors.yolo import YOLOv3
    from videotofaces.detection import normalize_detout
    from videotofaces.encoders.facenet import InceptionResnetV1
    from videotofaces.detection import boxes_to_crops

    B = args.det_batch
    pool_n = max(B, args.pool // B * B)
    frames_np = synth.make_frames(pool_n, H, W, seed=1000 + rank)
    frames = torch.from_numpy(frames_np).to(dev)
    yolo = args.det_model == 'yolo'
    # `lanes` independent (detector, encoder, HIP stream) sets work on alternate det-batches
    # from host threads (the ctypes calls release the GIL): one lane's host syncs and small
    # stage-2/3 kernels overlap the other lane's pyramid kernel.  Batches stay whole and
    # independent, so per-batch results are exactly the single-lane results.
    L = max(1, args.lanes)
    dets = [YOLOv3(dev, precision=args.det_precision) if yolo else MTCNN(dev) for _ in range(L)]
    if args.enc_model == 'facenet':
        encs = [InceptionResnetV1(dev, precision=args.enc_precision) for _ in range(L)]
        D = 512
    else:
        from videotofaces.encoders.vit import ViT
        vp = synth.make_params(args.enc_model)
        encs = [ViT(dev, vp, isL=args.enc_model == 'vit_l',
                    precision='fp32' if args.enc_precision == 'fp32' else 'f16x') for _ in range(L)]
        D = encs[0].dim
    streams = [torch.cuda.Stream(dev) for _ in range(L)]
    torch.cuda.synchronize(dev)

    def detect_step(lane, i):
        """one det-batch: detect + box post-processing -> crops with frame indices into the
        resident frame pool (so faces of consecutive det-batches can share encoder batches)."""
        j = (i * B) % pool_n
        fb = frames[j:j + B]
        res = normalize_detout(dets[lane](fb)) if yolo else dets[lane](fb, args.min_face_size)
        return boxes_to_crops(res, (H, W), frame_offset=j, **det_params(args)), sum(r.shape[0] for r in res)

    def run(first, n):
        """steps first..first+n-1, step i on lane i % L.  Each lane feeds its face stream to its
        encoder in batches of exactly enc_batch (encode_faces, grouping.py:29-40), flushing the
        remainder at the end.  Returns per-step (n faces, n detections) and the embeddings in
        global (step, face) order."""
        stats = [None] * n
        lane_embs = [[] for _ in range(L)]
        errs = []

        def lane_fn(lane):
            try:
                with torch.cuda.stream(streams[lane]):
                    pend = []
                    for k in range(lane, n, L):
                        crops, nd = detect_step(lane, first + k)
                        stats[k] = (crops.shape[0], nd)
                        pend.extend(crops.tolist())
                        while len(pend) >= args.enc_batch:
                            lane_embs[lane].append(encs[lane].encode_crops(frames, pend[:args.enc_batch]))
                            pend = pend[args.enc_batch:]
                    if pend:
                        lane_embs[lane].append(encs[lane].encode_crops(frames, pend))
            except BaseException as e:  # surfaced after join
                errs.append(e)
        ths = [threading.Thread(target=lane_fn, args=(l,)) for l in range(L)]
        for t in ths:
            t.start()
        for t in ths:
            t.join()
        if errs:
            raise errs[0]
        for s in streams:
            s.synchronize()
        # lane streams -> global (step, face) order
        parts, offs = [], [0] * L
        flat = [torch.cat(e) if e else torch.zeros((0, D), device=dev) for e in lane_embs]
        for k in range(n):
            lane, nf = k % L, stats[k][0]
            parts.append(flat[lane][offs[lane]:offs[lane] + nf])
            offs[lane] += nf
        return stats, parts

    run(0, max(args.warmup, L))
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    for d in dets:
        d.profile(True)
    t0 = time.perf_counter()
    stats, embs = run(args.warmup, args.steps)
    faces = sum(s_[0] for s_ in stats)
    dets_n = sum(s_[1] for s_ in stats)
    local_emb = torch.cat(embs) if embs else torch.zeros((0, D), device=dev)
    if world > 1:
        from videotofaces.parallel import all_gather_rows
        gathered = all_gather_rows(local_emb)
    else:
        gathered = local_emb
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    k_ms = k_launches = k_flops = k_frames = 0
    for d in dets:
        a, b_, c, e = d.profile(False)
        k_ms, k_launches, k_flops, k_frames = k_ms + a, k_launches + b_, k_flops + c, k_frames + e
    # the same kernel with the chip to itself (outside the timed region): one lane, 3 det-batches.
    # Under concurrent lanes the events above also span co-running kernels of the other lanes.
    dets[0].profile(True)
    with torch.cuda.stream(streams[0]):
        for i in range(3):
            detect_step(0, i)
    streams[0].synchronize()
    s_ms, s_launches, s_flops, _ = dets[0].profile(False)
    dets = dets_n
    tot = torch.tensor([faces, dets, k_frames], dtype=torch.float64, device=dev)
    el = torch.tensor([elapsed], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(tot, op=dist.ReduceOp.SUM)
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    faces_all, dets_all, frames_all = [float(x) for x in tot.tolist()]
    elapsed = float(el.item())
    if rank == 0:
        avg_ms = k_ms / max(1, k_launches)
        flops_per_launch = k_flops / max(1, k_launches)
        achieved = flops_per_launch / (avg_ms / 1e3) / 1e12 if avg_ms > 0 else 0.0
        traffic = None
        s_avg = s_ms / max(1, s_launches)
        s_ach = s_flops / max(1, s_launches) / (s_avg / 1e3) / 1e12 if s_avg > 0 else 0.0
        tf = os.path.join(ROOT, 'profiles', ('yolo' if yolo else 'pnet') + '_traffic.json')
        if os.path.exists(tf):
            traffic = json.load(open(tf)).get('hbm_bytes_per_launch')
        if yolo:
            peak = BF16_PEAK_TFLOPS if args.det_precision == 'bf16' else FP32_PEAK_TFLOPS
            kname = 'k_conv (YOLOv3 Darknet53+neck+head, 75 implicit-GEMM launches per det-batch, %s)' % args.det_precision
            wl = 'YOLOv3(%s)+%s' % (args.det_precision, ENC_NAMES[args.enc_model])
        else:
            peak = F16X_PEAK_TFLOPS
            kname = ('k_pnet (fused pyramid resample + PNet; convs on fp16 matrix cores with split operands, '
                     'fp32-grade; peak = fp16 dense / 3 products)')
            wl = 'MTCNN(min_face_size=%g)+%s' % (args.min_face_size, ENC_NAMES[args.enc_model])
        out = {
            'metric': 'faces/sec end-to-end (detect+encode) on %dx%d synthetic frames' % (W, H),
            'value': round(faces_all / elapsed, 2),
            'unit': 'faces/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': round(elapsed * 1e3 / args.steps, 3),
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': None,
            'dtype': '%s det / %s enc' % (args.det_precision if yolo else 'fp32 (split-fp16 MFMA)',
                                          args.enc_precision if args.enc_model == 'facenet' or args.enc_precision == 'fp32'
                                          else 'fp32 (split-fp16 MFMA)'),
            'data': 'synthetic (seeded %s value-noise frames with face blobs; hash-seeded synthetic weights, '
                    'detector heads calibrated to a few faces/frame)' % args.frame,
            'config': {'workload': '%s, det-batch %d, enc-batch %d, %s, frames in HBM, '
                                   'box filter min_score %g min_size %d min_border %d, det_scale (1.5,1.5,2.2,1.2), square'
                                   % (wl, B, args.enc_batch, args.frame, args.det_min_score, args.det_min_size,
                                      args.det_min_border),
                       'det_batch': B, 'enc_batch': args.enc_batch, 'frames_per_step_per_gpu': B,
                       'lanes': L,
                       'parallelism': 'dp%d (frame-sharded, RCCL all-gather of embeddings)' % world},
            'frames_per_s': round(world * args.steps * B / elapsed, 2),
            'faces_per_frame': round(faces_all / max(1.0, world * args.steps * B), 3),
            'detections_per_frame': round(dets_all / max(1.0, world * args.steps * B), 3),
            'roofline': {'kernel': kname, 'bound': 'mfma',
                         'achieved': round(achieved, 3), 'peak': peak, 'unit': 'TFLOP/s',
                         'frac': round(achieved / peak, 4), 'traffic': traffic,
                         'avg_launch_ms': round(avg_ms, 4), 'flops_per_launch': flops_per_launch,
                         'launches': k_launches, 'concurrent_lanes': L,
                         'solo': {'avg_launch_ms': round(s_avg, 4), 'achieved': round(s_ach, 3),
                                  'frac': round(s_ach / peak, 4), 'launches': s_launches}},
            # north-star's "memory-bound HBM roofline on the detector conv path": the layer-by-layer
            # PNet bytes of SURVEY.md §8d (2,075 MB fp32 per 720p frame at 38.66 GFLOP, AI 18.6) over
            # the same launch time -- an equivalent rate (the fused kernel moves `traffic` bytes)
            'hbm_equiv': None if yolo else {
                'bytes_per_launch': round(flops_per_launch * LBL_BYTES_PER_FLOP),
                'achieved': round(flops_per_launch * LBL_BYTES_PER_FLOP / (avg_ms / 1e3) / 1e9, 1) if avg_ms > 0 else 0.0,
                'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                'frac': round(flops_per_launch * LBL_BYTES_PER_FLOP / (avg_ms / 1e3) / 1e9 / HBM_PEAK_GBS, 4)
                if avg_ms > 0 else 0.0,
                'solo_frac': round(s_flops / max(1, s_launches) * LBL_BYTES_PER_FLOP / (s_avg / 1e3) / 1e9
                                   / HBM_PEAK_GBS, 4) if s_avg > 0 else 0.0},
            'cpu_baseline': None,
        }
        if world == 1 and not args.no_cpu_baseline:
            out['cpu_baseline'] = cpu_baseline(frames_np, args)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()

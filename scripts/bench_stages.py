"""Stage benches beside bench.py's headline line: one JSON line per stage.

  vit       BASELINE config 4: ViT-L/16 (or -B) encoder-only, enc-batch 128 over pre-cropped
            224x224 uint8 faces resident in HBM (blob 224 -> 128 + ViT forward; split-fp16 or fp32 MFMA);
            roofline = encoder FLOPs (39.78 / 11.27 GFLOP per face) / step time.
  grouping  the grouping step on N planted-cluster embeddings (N=10k, D=512 by default):
            fused cosine dedupe (dupes.py:51-68) and the KMeans + silhouette/CH/DB sweep
            (grouping.py:92-137) for k = 2..16, each timed with a device sync on both sides.

The CPU legs are the oracle (ViT torch-CPU restatement) and sklearn 1.7.2 itself (the
reference's own grouping dependency), on bounded samples, timed on this host's cores.

  python scripts/bench_stages.py vit [--vit-model vit_l] [--steps 10] [--warmup 2]
  python scripts/bench_stages.py grouping [--n 10000] [--d 512]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'video-to-faces_amd')]

import numpy as np  # noqa: E402
import torch  # noqa: E402

FP32_PEAK_TFLOPS = 157.3  # MI355X dense fp32 MFMA (MI355X_MICROARCH.md)
F16X_PEAK_TFLOPS = round(2500.0 / 3, 1)  # fp16 dense MFMA / 3 products (split-fp16 operands)
VIT_GFLOP = {'vit_b': 11.27, 'vit_l': 39.78}  # per face at 128x128


def cores():
    n = len(os.sched_getaffinity(0))
    env = os.environ.get('OMP_NUM_THREADS')
    return min(n, int(env)) if env and env.isdigit() else n


def bench_vit(a):
    from videotofaces import synth
    from videotofaces.encoders.vit import ViT
    isL = a.vit_model == 'vit_l'
    dev = torch.device('cuda:0')
    params = synth.make_params(a.vit_model)
    m = ViT(dev, params, isL=isL, precision=a.vit_precision)
    B = a.enc_batch
    crops_u8 = torch.from_numpy(synth.make_crops(B, 224, seed=1)).to(dev)  # [B,224,224,3] in HBM
    boxes = np.array([[i, 0, 0, 224, 224] for i in range(B)], np.int32)
    stream = torch.cuda.current_stream(dev)
    for _ in range(a.warmup):
        m.encode_crops(crops_u8, boxes)
    torch.cuda.synchronize(dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    e0.record(stream)
    for _ in range(a.steps):
        out = m.encode_crops(crops_u8, boxes)
    e1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t0
    ms = e0.elapsed_time(e1) / a.steps
    assert out.shape == (B, m.dim) and bool(torch.isfinite(out).all())
    achieved = VIT_GFLOP[a.vit_model] * B / ms  # GFLOP/ms = TFLOP/s
    # split-fp16: three fp16 products per fp32-grade product -> fp16 dense peak / 3
    peak = FP32_PEAK_TFLOPS if a.vit_precision == 'fp32' else F16X_PEAK_TFLOPS
    res = {'metric': 'faces/sec, %s encoder on pre-cropped 224x224 faces (BASELINE config 4)' % a.vit_model,
           'value': round(a.steps * B / wall, 2), 'unit': 'faces/s', 'n_gpus': 1, 'steps': a.steps,
           'warmup': a.warmup, 'ms_per_step': round(wall * 1e3 / a.steps, 3), 'higher_is_better': True,
           'dtype': 'fp32' if a.vit_precision == 'fp32' else 'fp32 (split-fp16 MFMA, guarded)', 'data': 'synthetic (seeded 224x224 crops, hash-seeded weights)',
           'config': {'workload': '%s enc-batch %d, 224x224 uint8 crops in HBM -> blob 128x128 -> ViT'
                                  % (a.vit_model, B), 'enc_batch': B},
           'roofline': {'kernel': 'whole encoder step (blob + %d k_conv GEMM launches + attention + LN)'
                                  % (12 * (2 if isL else 1) * 4 + 2),
                        'bound': 'mfma', 'achieved': round(achieved, 3), 'peak': peak,
                        'unit': 'TFLOP/s', 'frac': round(achieved / peak, 4),
                        'gflop_per_face': VIT_GFLOP[a.vit_model], 'event_ms_per_step': round(ms, 3)},
           'cpu_baseline': None}
    if not a.no_cpu_baseline:
        from oracle.vit import vit
        torch.set_num_threads(cores())
        n = a.cpu_faces
        x = (torch.from_numpy(synth.make_crops(n, 128, seed=2)).permute(0, 3, 1, 2).float() - 127.5) / 127.5
        dim, depth = (1024, 24) if isL else (768, 12)
        vit(params, x[:1], dim, depth)  # warm-up
        t0 = time.time()
        vit(params, x, dim, depth)
        dt = time.time() - t0
        res['cpu_baseline'] = {'value': round(n / dt, 3), 'unit': 'faces/s', 'cores': cores(), 'kind': 'port',
                               'sample': '%d faces at 128x128, oracle %s forward fp32 on CPU, %.1f s'
                                         % (n, a.vit_model, dt)}
    print(json.dumps(res), flush=True)


def bench_grouping(a):
    from videotofaces import synth, dupes
    from videotofaces.grouping import cluster_sweep
    dev = torch.device('cuda:0')
    X = synth.planted_clusters(a.n, a.d, seed=0)
    Xd = torch.from_numpy(X).to(dev)
    ks = list(range(2, a.kmax + 1))
    dupes.cosine_dedupe_device(Xd[:256])  # warm-up (library load, scratch)
    cluster_sweep(X[:512], [2], 0)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    mins, inds = dupes.cosine_dedupe_device(Xd)
    torch.cuda.synchronize(dev)
    t_dd = time.perf_counter() - t0
    t0 = time.perf_counter()
    labels, scores = cluster_sweep(X, ks, 0)
    torch.cuda.synchronize(dev)
    t_sw = time.perf_counter() - t0
    best_k = scores[int(np.argmax([s[1] for s in scores]))][0]
    cos_tflop = a.n * a.n * a.d / 1e12  # lower-triangle GEMM, 2 FLOP per MAC
    res = {'metric': 'grouping time (cosine dedupe + KMeans/silhouette/CH/DB sweep k=2..%d)' % a.kmax,
           'value': round(t_dd + t_sw, 4), 'unit': 's', 'higher_is_better': False, 'n_gpus': 1,
           'dtype': 'fp32 (KMeans bit-exact labels, scores f64)',
           'data': 'synthetic planted clusters (8 centres, sigma 0.5, seed 0)',
           'config': {'workload': 'N=%d D=%d' % (a.n, a.d), 'N': a.n, 'D': a.d, 'k': [ks[0], ks[-1]]},
           'dedupe_s': round(t_dd, 4), 'sweep_s': round(t_sw, 4), 'sweep_s_per_k': round(t_sw / len(ks), 4),
           'best_k_silhouette': int(best_k), 'dupes_at_0.25': int((mins <= 0.25).sum()),
           'dedupe_roofline': {'bound': 'mfma', 'achieved': round(cos_tflop / t_dd, 3), 'peak': FP32_PEAK_TFLOPS,
                               'unit': 'TFLOP/s', 'frac': round(cos_tflop / t_dd / FP32_PEAK_TFLOPS, 4)},
           'cpu_baseline': None}
    if not a.no_cpu_baseline:
        import sklearn.cluster
        import sklearn.metrics
        from oracle import grouping as og
        torch.set_num_threads(cores())
        t0 = time.time()
        og.cosine_dedupe(X)
        c_dd = time.time() - t0
        kc = ks[:a.cpu_ks]
        t0 = time.time()
        for k in kc:
            lb = sklearn.cluster.KMeans(n_clusters=k, random_state=0, n_init='auto').fit_predict(X)
            sklearn.metrics.silhouette_score(X, lb)
            sklearn.metrics.calinski_harabasz_score(X, lb)
            sklearn.metrics.davies_bouldin_score(X, lb)
        c_k = (time.time() - t0) / len(kc)
        res['cpu_baseline'] = {'value': round(c_dd + c_k * len(ks), 3), 'unit': 's', 'cores': cores(),
                               'kind': 'reference',
                               'sample': 'sklearn 1.7.2 (the reference\'s grouping dependency): cosine dedupe '
                                         '%.2f s at N=%d + %.2f s per k measured on k=%s, scaled to %d k'
                                         % (c_dd, a.n, c_k, kc, len(ks))}
    print(json.dumps(res), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('stage', choices=['vit', 'grouping'])
    ap.add_argument('--vit-model', default='vit_l', choices=['vit_b', 'vit_l'])
    ap.add_argument('--vit-precision', default='f16x', choices=['fp32', 'f16x'])
    ap.add_argument('--enc-batch', type=int, default=128)
    ap.add_argument('--steps', type=int, default=10)
    ap.add_argument('--warmup', type=int, default=2)
    ap.add_argument('--cpu-faces', type=int, default=16)
    ap.add_argument('--n', type=int, default=10000)
    ap.add_argument('--d', type=int, default=512)
    ap.add_argument('--kmax', type=int, default=16)
    ap.add_argument('--cpu-ks', type=int, default=3)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    a = ap.parse_args()
    bench_vit(a) if a.stage == 'vit' else bench_grouping(a)


if __name__ == '__main__':
    main()

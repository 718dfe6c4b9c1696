"""CPU-twin calibration (the timed twin within +-15 % of the reference modules).

Runs in the survey container only (the reference imports there through the import shims of
tests/golden/make_golden.py; it never travels to the GPU box).  For each stage the reference's
own nn.Module and the oracle restatement (oracle/*.py, the code bench.py's cpu_baseline times)
run on the same seeded frames / blobs with the same synthetic weights, warm-up 1 + min of 5
repeats, torch threads = the cores used.  Writes profiles/<tag>_cpu_twin_calibration.json.

    python scripts/calibrate_cpu_twin.py [tag]
"""
import importlib
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'video-to-faces_amd'), os.path.join(ROOT, 'tests', 'golden')]
import make_golden as mg  # noqa: E402
from videotofaces import synth  # noqa: E402
from oracle import mtcnn as om, facenet as ofn, yolo as oy, vit as ovit  # noqa: E402


def tpair(fa, fb, reps=5):
    """min-of-reps wall time of fa and fb, measured alternately (a drift in the host's speed
    hits both sides alike)"""
    fa(), fb()
    best = [1e30, 1e30]
    for _ in range(reps):
        for i, fn in enumerate((fa, fb)):
            t0 = time.perf_counter()
            fn()
            best[i] = min(best[i], time.perf_counter() - t0)
    return best


def main(tag):
    cores = len(os.sched_getaffinity(0))
    torch.set_num_threads(cores)
    mg.load_ref()
    # the shim's torchvision NMS (make_golden._tv_nms) is a Python loop, far slower than
    # torchvision's C++ kernel; for timing, the shimmed reference calls the C restatement of that
    # kernel (oracle/nms_oracle.c), as the twin does
    from oracle import nms as onms
    sys.modules['torchvision.ops'].batched_nms = onms.batched_nms
    sys.modules['torchvision.ops'].nms = onms.nms
    rows = []

    def row(stage, unit, n, fa, fb):
        t_ref, t_twin = tpair(fa, fb)
        r = {'stage': stage, 'unit': unit, 'units': n, 'ref_s_per_unit': t_ref / n,
             'twin_s_per_unit': t_twin / n, 'twin_over_ref': t_twin / t_ref,
             'within_15pct': abs(t_twin / t_ref - 1) <= 0.15}
        rows.append(r)
        print(json.dumps(r), flush=True)

    # MTCNN full detector forward, det-batch 1 (config 1), RealMTCNN min_face_size 5
    m = importlib.import_module('ref_vtf.detectors.mtcnn')
    pm = synth.make_params('mtcnn')
    net = mg._load(m.MTCNN('cpu'), pm)
    frames = synth.make_frames(2, seed=0)

    def ref_mtcnn():
        with torch.inference_mode():
            for f in range(frames.shape[0]):
                net(list(frames[f:f + 1]), 5)

    def twin_mtcnn():
        for f in range(frames.shape[0]):
            om.forward(pm, list(frames[f:f + 1]), minsize=5)
    row('MTCNN forward, det-batch 1, min_face_size 5, 720p', 'frame', frames.shape[0], ref_mtcnn, twin_mtcnn)

    # FaceNet (InceptionResnetV1, 160^2) batch 16
    f = importlib.import_module('ref_vtf.encoders.facenet')
    pf = synth.make_params('facenet')
    fnet = mg._load(f.InceptionResnetV1('cpu'), pf)
    u8 = torch.from_numpy(mg._u8(103, (16, 3, 160, 160)))
    x = (u8.float() - 127.5) * (1 / 128)

    def ref_fn():
        with torch.inference_mode():
            fnet(x)
    row('FaceNet forward, batch 16', 'face', 16, ref_fn, lambda: ofn.inception_resnet_v1(pf, x))

    # YOLOv3 backbone + neck + head on the 608 letterbox of 720p frames, batch 1
    y = importlib.import_module('ref_vtf.detectors.yolo')
    py = synth.make_params('yolo')
    ynet = mg._load(y.YOLOv3('cpu'), py)
    yx, _, _, _ = mg._yolo_input(list(synth.make_frames(1, seed=1)))

    def ref_y():
        with torch.inference_mode():
            ynet.head(ynet.neck(ynet.backbone(yx)))
    row('YOLOv3 net, batch 1, 720p letterbox %dx%d' % tuple(yx.shape[-2:]), 'frame', 1,
        ref_y, lambda: oy.net(py, yx))

    # ViT-L/16 (128^2, 65 tokens) batch 16
    v = importlib.import_module('ref_vtf.encoders.vit')
    pv = synth.make_params('vit_l')
    vnet = mg._load(v.ViT('cpu', 128, 16, 1024, 24), pv)
    u8 = torch.from_numpy(mg._u8(104, (16, 3, 128, 128)))
    xv = (u8.float() - 127.5) * np.float32(1 / 127.5)

    def ref_v():
        with torch.inference_mode():
            vnet(xv)
    row('ViT-L/16 forward, batch 16', 'face', 16, ref_v, lambda: ovit.vit(pv, xv, 1024, 24))

    out = {'cores': cores, 'torch_threads': torch.get_num_threads(), 'torch': torch.__version__,
           'nms': 'torchvision batched_nms in the shimmed reference = the C restatement oracle/nms_oracle.c (timing only)',
           'protocol': 'warm-up 1, min of 5 repeats taken alternately (reference, twin), same seeded inputs and synthetic weights',
           'rows': rows, 'all_within_15pct': all(r['within_15pct'] for r in rows)}
    path = os.path.join(ROOT, 'profiles', '%s_cpu_twin_calibration.json' % tag)
    with open(path, 'w') as fh:
        json.dump(out, fh, indent=1)
    print('wrote', path, 'all within 15%:', out['all_within_15pct'])


if __name__ == '__main__':
    main(sys.argv[1] if len(sys.argv) > 1 else 'r02r')

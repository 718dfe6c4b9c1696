"""Time vtf_batched_nms (csrc/nms.hip) on MTCNN-like candidate sets: B images, clusters of
jittered boxes around face positions at several sizes plus scattered background boxes.

    python scripts/nms_time.py [reps]
"""
import ctypes
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'video-to-faces_amd')]
from videotofaces import _native as nat  # noqa: E402


def candidates(n, B, thr_seed=0):
    rng = np.random.default_rng(thr_seed)
    img = rng.integers(0, B, n)
    centers = rng.uniform(50, 1200, (B, 12, 2))
    sizes = rng.uniform(12, 200, (B, 12))
    k = rng.integers(0, 12, n)
    cl = rng.random(n) < 0.8
    c = centers[img, k] + rng.normal(0, 1, (n, 2)) * sizes[img, k, None] * 0.15
    s = sizes[img, k] * np.exp(rng.normal(0, 0.2, n))
    bg = ~cl
    c[bg] = rng.uniform(0, 1280, (bg.sum(), 2))
    s[bg] = rng.uniform(12, 100, bg.sum())
    boxes = np.stack([c[:, 0] - s / 2, c[:, 1] - s / 2, c[:, 0] + s / 2, c[:, 1] + s / 2], 1).astype(np.float32)
    scores = rng.random(n).astype(np.float32)
    return boxes, scores, img.astype(np.int64)


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    lib = nat.lib()
    st = torch.cuda.current_stream().cuda_stream
    for n, thr in ((38000, 0.5), (20000, 0.7), (8000, 0.7), (2000, 0.5)):
        boxes, scores, img = candidates(n, 16)
        db, ds, di = (torch.from_numpy(x).cuda() for x in (boxes, scores, img))
        keep = torch.empty(n, dtype=torch.int64, device='cuda')
        nk = ctypes.c_int64(0)
        ts = []
        for r in range(reps + 3):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            rc = lib.vtf_batched_nms(db.data_ptr(), ds.data_ptr(), di.data_ptr(), n, thr, keep.data_ptr(),
                                     ctypes.byref(nk), st)
            torch.cuda.synchronize()
            ts.append(time.perf_counter() - t0)
            assert rc == 0
        print('n %d thr %.1f: kept %d, host-timed %.3f ms (median of %d)' % (n, thr, nk.value, 1e3 * np.median(ts[3:]), reps),
              flush=True)


if __name__ == '__main__':
    main()

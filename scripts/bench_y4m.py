"""Measure the .y4m frame source (videotofaces/video.py + csrc/video.hip): the conversion
kernel on resident planes (HIP events on its stream; algorithmic bytes = 1.5 B read + 3 B written
per 4:2:0 pixel) and the whole read() of a det-batch of 16 sampled 720p frames from a file in the
page cache (gather into pinned memory + H2D + kernel).  python scripts/bench_y4m.py [out.json]"""
import json
import os
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..', 'video-to-faces_amd'))
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), '..'))


def main():
    from videotofaces import _native as nat
    from videotofaces.video import Y4MReader
    H, W, B = 720, 1280, 16
    fb = H * W * 3 // 2
    rng = np.random.default_rng(0)
    dev = torch.device('cuda:0')
    st = torch.cuda.current_stream(dev)
    planes = torch.from_numpy(rng.integers(0, 256, (B, fb), dtype=np.uint8)).to(dev)
    out = torch.empty((B, H, W, 3), dtype=torch.uint8, device=dev)

    def conv():
        nat.check(nat.lib().vtf_yuv_to_bgr(nat.ptr(planes), B, H, W, 420, 0, fb, nat.ptr(out), out.stride(0),
                                           out.stride(1), nat.stream_ptr(dev)))
    for _ in range(20):
        conv()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 200
    e0.record(st)
    for _ in range(n):
        conv()
    e1.record(st)
    torch.cuda.synchronize()
    k_ms = e0.elapsed_time(e1) / n
    bytes_per_launch = B * H * W * 4.5
    res = {'kernel': 'k_yuv420_to_bgr_8x2<false>', 'frames_per_launch': B, 'size': [H, W],
           'avg_launch_us': k_ms * 1e3, 'achieved_GBps': bytes_per_launch / (k_ms * 1e-3) / 1e9, 'peak_GBps': 8000,
           'bytes_per_launch': bytes_per_launch}
    res['frac'] = res['achieved_GBps'] / res['peak_GBps']
    # the whole read() of 16 sampled frames (step 2) from a 64-frame file in the page cache
    from videotofaces.video import write_y4m
    with tempfile.TemporaryDirectory() as d:
        f = os.path.join(d, 'clip.y4m')
        write_y4m(f, rng.integers(0, 256, (64, fb), dtype=np.uint8), H, W, fps='30:1')
        r = Y4MReader(f)
        idx = list(range(1, 64, 4))[:B]
        for _ in range(3):
            r.read(idx)
        torch.cuda.synchronize()
        reps = 20
        t0 = time.perf_counter()
        for _ in range(reps):
            r.read(idx)
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / reps
        r.close()
    res['read_ms_per_det_batch'] = dt * 1e3
    res['read_frames_per_s'] = B / dt
    res['read_note'] = 'page-cache file -> pinned gather -> one H2D of 1.5 B/px -> kernel, synchronous per batch'
    line = json.dumps(res)
    print(line)
    if len(sys.argv) > 1:
        with open(sys.argv[1], 'w') as fh:
            fh.write(line + '\n')


if __name__ == '__main__':
    main()

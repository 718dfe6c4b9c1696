"""YOLOv3 (x3) detect on 32 distinct 720p frames under env modes (interleaved rounds, one process):
the detections of every mode compared with the first mode's, and the time per det-batch.

    python scripts/r06_yolo_ab.py reps MODE[,MODE...]   (MODE = NAME=V[+NAME=V...])
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'video-to-faces_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def flatten(o):
    if isinstance(o, (list, tuple)):
        return [v for x in o for v in flatten(x)]
    if isinstance(o, torch.Tensor):
        o = o.cpu().numpy()
    return list(np.asarray(o, dtype=np.float64).ravel())


def main():
    from videotofaces.detectors.yolo import YOLOv3
    from videotofaces import synth
    reps = int(sys.argv[1])
    modes = sys.argv[2].split(',')
    det = YOLOv3('cuda:0', precision='x3')
    frames = synth.make_frames_device(0, 32, 720, 1280, seed=5, device='cuda:0', style='blobs')

    def setenv(mode):
        for kv in mode.split('+'):
            k, v = kv.split('=')
            os.environ[k] = v
    res, ref = {}, None
    for rnd in range(4):
        for mode in modes:
            setenv(mode)
            out = det(frames)
            torch.cuda.synchronize()
            if rnd == 0:
                flat = np.asarray(flatten(out), dtype=np.float64)
                if ref is None:
                    ref = flat
                print('%s: detections identical to %s: %s (%d values)' % (mode, modes[0], bool(np.array_equal(flat, ref)), flat.size), flush=True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                det(frames)
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(mode, []).append(e0.elapsed_time(e1) / reps)
    for mode, v in res.items():
        print('%s: det-batch of 32 %s ms' % (mode, ' '.join('%.3f' % t for t in v)), flush=True)


if __name__ == '__main__':
    main()

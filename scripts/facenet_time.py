"""Time the FaceNet bf16 forward at enc-batch 128 (HIP events on the encoder's stream), fused
Block17 vs the unfused launches (VTF_FN_FUSED), interleaved in one process.

    python scripts/facenet_time.py [reps]
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'video-to-faces_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    from videotofaces.encoders.facenet import InceptionResnetV1
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    # modes: comma-separated; a mode is '1' / '0' (VTF_FN_FUSED) or NAME=V[+NAME=V...] env settings
    modes = sys.argv[2].split(',') if len(sys.argv) > 2 else ['1', '0']
    m = InceptionResnetV1('cuda:0', precision='bf16')
    u8 = torch.from_numpy(np.random.default_rng(0).integers(0, 256, (128, 3, 160, 160), dtype=np.uint8))
    x = ((u8.float() - 127.5) * (1 / 128)).cuda()
    res = {}
    for rnd in range(3):
        for mode in modes:
            for kv in (mode.split('+') if '=' in mode else ['VTF_FN_FUSED=' + mode]):
                k, v = kv.split('=')
                os.environ[k] = v
            m(x)
            torch.cuda.synchronize()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                m(x)
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(mode, []).append(e0.elapsed_time(e1) / reps)
    for mode, v in res.items():
        print('%s: forward per 128 faces %s ms' % (mode if '=' in mode else 'VTF_FN_FUSED=' + mode,
                                                   ' '.join('%.3f' % t for t in v)))


if __name__ == '__main__':
    main()

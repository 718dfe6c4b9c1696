"""Encoder forward per 128 faces under env modes (interleaved rounds, one process), with the
embeddings of every mode compared bit for bit with the first mode's.

    python scripts/r06_b17ws.py reps MODE[,MODE...] [facenet|vit_l]   (MODE = NAME=V[+NAME=V...])
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'video-to-faces_amd')]
import numpy as np  # noqa: E402
import torch  # noqa: E402


def main():
    reps = int(sys.argv[1])
    modes = sys.argv[2].split(',')
    model = sys.argv[3] if len(sys.argv) > 3 else 'facenet'
    def make():
        if model == 'facenet':
            from videotofaces.encoders.facenet import InceptionResnetV1
            return InceptionResnetV1('cuda:0', precision='bf16'), 160
        from videotofaces.encoders.vit import ViT
        return ViT('cuda:0', isL=model == 'vit_l', precision='f16x'), 128

    def setenv(mode):
        for kv in mode.split('+'):
            k, v = kv.split('=')
            os.environ[k] = v
    # one model per mode, built under the mode's env (build-time switches such as VTF_FN_WPAD)
    models = {}
    for mode in modes:
        setenv(mode)
        models[mode], side = make()
    u8 = torch.from_numpy(np.random.default_rng(0).integers(0, 256, (128, 3, side, side), dtype=np.uint8))
    x = ((u8.float() - 127.5) * (1 / 128)).cuda()
    res, ref = {}, None
    for rnd in range(4):
        for mode in modes:
            setenv(mode)
            m = models[mode]
            e = m(x)
            torch.cuda.synchronize()
            if rnd == 0:
                e = e.cpu().numpy() if hasattr(e, 'cpu') else np.asarray(e)
                if ref is None:
                    ref = e
                print('%s: embeddings identical to %s: %s' % (mode, modes[0], bool(np.array_equal(e, ref))), flush=True)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(reps):
                m(x)
            e1.record()
            torch.cuda.synchronize()
            res.setdefault(mode, []).append(e0.elapsed_time(e1) / reps)
    for mode, v in res.items():
        print('%s: forward per 128 faces %s ms' % (mode, ' '.join('%.3f' % t for t in v)), flush=True)


if __name__ == '__main__':
    main()

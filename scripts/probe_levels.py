"""Per-pyramid-level timing of the fused resample+PNet kernel (dense parity entry point)."""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'video-to-faces_amd')]
import torch
from videotofaces import synth
from videotofaces.detectors.mtcnn import MTCNN
from oracle.mtcnn import scale_pyramid
fr = torch.from_numpy(synth.make_frames(16, seed=0)).cuda()
m = MTCNN('cuda:0')
scales, sizes = scale_pyramid(720, 1280, 5)
tot = 0
for i, (lh, lw) in enumerate(sizes):
    m.pnet_level(fr, lh, lw)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(3):
        m.pnet_level(fr, lh, lw)
    e1.record(); torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 3
    ph, pw = (lh - 1) // 2 - 4, (lw - 1) // 2 - 4
    tiles = 16 * -(-ph // 16) * -(-pw // 32)
    tot += ms
    print('level %2d %4dx%4d scale %.3f tiles %6d  %.3f ms  %.2f us/tile' % (i, lh, lw, scales[i], tiles, ms, ms * 1e3 / tiles))
print('sum %.3f ms' % tot)

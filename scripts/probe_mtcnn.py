"""Timing probe: MTCNN detect on det-batch of 720p frames resident in HBM."""
import os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'video-to-faces_amd')]
import numpy as np, torch
from videotofaces import synth
from videotofaces.detectors.mtcnn import MTCNN
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 5
fr = torch.from_numpy(synth.make_frames(B, seed=0)).cuda()
m = MTCNN('cuda:0')
res = m(fr, 5); torch.cuda.synchronize()
print('stats', m.last_stats.tolist(), 'faces', sum(r.shape[0] for r in res))
t = time.time()
for _ in range(iters):
    res = m(fr, 5)
torch.cuda.synchronize()
dt = (time.time() - t) / iters
print('B=%d  %.2f ms/batch  %.3f ms/frame  %.1f frames/s  %.1f faces/s' % (B, dt * 1e3, dt * 1e3 / B, B / dt, sum(r.shape[0] for r in res) / dt))

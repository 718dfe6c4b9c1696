"""Stage counts of MTCNN on the bench's synthetic det-batches (k1..k3 = boxes entering the next
stage): python scripts/mtcnn_stats.py [batches]"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'video-to-faces_amd')]
import numpy as np
import torch
from videotofaces import synth
from videotofaces.detectors.mtcnn import MTCNN
n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
frames = torch.from_numpy(synth.make_frames(16 * n, seed=1000)).cuda()
m = MTCNN('cuda:0')
names = ['levels', 'stage1 cand', 'after lvl nms', 'rnet in', 'rnet pass', 'onet in', 'onet pass', 'final']
acc = np.zeros(8, np.int64)
for i in range(n):
    try:
        m(frames[16 * i:16 * i + 16], 5)
    except Exception as e:  # phase-skip probes produce garbage downstream
        print('error:', str(e)[:120])
        continue
    acc += m.last_stats
    print(dict(zip(names, m.last_stats.tolist())), flush=True)
print('mean per det-batch', dict(zip(names, (acc / n).round(1).tolist())))

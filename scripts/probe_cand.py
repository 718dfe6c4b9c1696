"""Run MTCNN on one det-batch of 16 synthetic 720p frames a few times; print the stage counts
(candidates into RNet = stats[3], into ONet = stats[5]) for per-candidate kernel times."""
import os
import sys
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'video-to-faces_amd')]
import torch  # noqa: E402
from videotofaces import synth  # noqa: E402
from videotofaces.detectors.mtcnn import MTCNN  # noqa: E402
fr = torch.from_numpy(synth.make_frames(16, seed=1000)).cuda()
m = MTCNN('cuda:0')
for _ in range(int(sys.argv[1]) if len(sys.argv) > 1 else 5):
    m(fr, 5)
torch.cuda.synchronize()
print('stats', m.last_stats.tolist())

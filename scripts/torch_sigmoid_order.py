"""Check oracle/rcnn.py's restatement of torch's CPU sigmoid (torch_sigmoid_survey: Sleef
expf u10 on vector steps, glibc expf on each parallel_for chunk's tail) -- which the device RPN
decode (rcnn.hip torch_sigmoid) follows -- against torch itself, bit for bit.

    python scripts/torch_sigmoid_order.py
"""
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, 'video-to-faces_amd')]
from oracle.rcnn import torch_sigmoid_survey  # noqa: E402


def main():
    print('torch', torch.__version__, 'cpu capability', torch.backends.cpu.get_cpu_capability(),
          'threads', torch.get_num_threads())
    rng = np.random.default_rng(0)
    x = rng.normal(0, 3, 400000).astype(np.float32)
    for n in (400000, 100000, 38048, 9512, 77):
        ref = torch.from_numpy(x[:n]).sigmoid().numpy()
        got = torch_sigmoid_survey(x[:n], torch.get_num_threads())
        print('n=%d: %d of %d differ' % (n, int((got != ref).sum()), n))


if __name__ == '__main__':
    main()

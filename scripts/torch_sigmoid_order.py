"""(1) Check oracle/rcnn.py's restatement of torch's CPU sigmoid (torch_sigmoid_survey: Sleef
expf u10 on vector steps, glibc expf on each parallel_for chunk's tail) -- which the device RPN
decode (rcnn.hip torch_sigmoid) follows -- against torch itself, bit for bit.  (2) Check that std::sort of (value, position) pairs with
ATen's KeyValueCompDesc -- what rcnn.hip uses for batched_nms's final unstable sort -- orders
ties exactly like torch.sort(descending=True) on CPU (g++ on the same libstdc++ algorithm).

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


SORT_CPP = r"""
#include <algorithm>
#include <cmath>
#include <utility>
#include <vector>
extern "C" void sort_desc(const float* v, long n, long* out) {
    std::vector<std::pair<float, long>> a(n);
    for (long i = 0; i < n; i++) a[i] = {v[i], i};
    std::sort(a.begin(), a.end(), [](const std::pair<float, long>& l, const std::pair<float, long>& r) {
        return (std::isnan(l.first) && !std::isnan(r.first)) || (l.first > r.first);
    });
    for (long i = 0; i < n; i++) out[i] = a[i].second;
}
"""


def check_sort():
    import ctypes
    import subprocess
    import tempfile
    d = tempfile.mkdtemp()
    open(os.path.join(d, 's.cpp'), 'w').write(SORT_CPP)
    subprocess.check_call(['g++', '-O2', '-shared', '-fPIC', os.path.join(d, 's.cpp'), '-o', os.path.join(d, 's.so')])
    lib = ctypes.CDLL(os.path.join(d, 's.so'))
    lib.sort_desc.argtypes = [ctypes.c_void_p, ctypes.c_long, ctypes.c_void_p]
    g = torch.Generator().manual_seed(0)
    ok = 0
    for n in (10, 17, 100, 1000, 2000, 5000, 20000):
        for levels in (3, 50):
            v = torch.randint(0, levels, (n,), generator=g).float().numpy()
            out = np.zeros(n, np.int64)
            lib.sort_desc(v.ctypes.data, n, out.ctypes.data)
            ok += np.array_equal(out, torch.from_numpy(v).sort(descending=True)[1].numpy())
    print('std::sort pairs == torch unstable sort on %d of 14 tie-heavy inputs' % ok)


if __name__ == '__main__':
    main()
    check_sort()

"""Steady-state dispatches per det-batch from a one-lane rocprofv3 kernel trace of bench.py.

  python scripts/dispatch_counts.py TRACE_DIR [anchor]

Counts every kernel dispatched after the first `anchor` kernel (default: the exact-levels k_pnet,
one per det-batch), so the model-build weight uploads and warm-up allocations are excluded, and
divides by the number of anchor dispatches: runtime blit copies (__amd_rocclr_copyBuffer), fills
(__amd_rocclr_fillBuffer*) and all dispatches per det-batch."""
import glob
import os
import sqlite3
import sys
from collections import Counter


def main():
    path = sys.argv[1]
    anchor = sys.argv[2] if len(sys.argv) > 2 else 'k_pnet<false, true'
    if os.path.isdir(path):
        path = glob.glob(os.path.join(path, '**', '*results.db'), recursive=True)[0]
    c = sqlite3.connect(path)
    cols = [r[1] for r in c.execute('pragma table_info(kernels)')]
    t0 = 'start' if 'start' in cols else [x for x in cols if 'start' in x][0]
    rows = c.execute('select name, %s from kernels order by %s' % (t0, t0)).fetchall()
    first = next((i for i, (n, _) in enumerate(rows) if anchor in n), None)
    if first is None:
        print('anchor %r not found' % anchor)
        return
    tail = rows[first:]
    nb = sum(1 for n, _ in tail if anchor in n)
    cnt = Counter()
    for n, _ in tail:
        if 'copyBuffer' in n:
            cnt['copyBuffer'] += 1
        elif 'fillBuffer' in n:
            cnt['fillBuffer'] += 1
        cnt['all'] += 1
    print('det-batches (anchor dispatches): %d' % nb)
    for k in ('copyBuffer', 'fillBuffer', 'all'):
        print('%-12s %7d total  %7.2f per det-batch' % (k, cnt[k], cnt[k] / max(nb, 1)))
    print('(whole trace: %d copyBuffer, %d fillBuffer of %d dispatches)' % (
        sum('copyBuffer' in n for n, _ in rows), sum('fillBuffer' in n for n, _ in rows), len(rows)))


if __name__ == '__main__':
    main()

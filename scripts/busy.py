"""GPU occupancy of a rocprofv3 kernel trace (results db): the union of kernel intervals over the
span from the first to the last kernel, and the share of that span each kernel class covers with
no other kernel running.  usage: busy.py db_dir [skip_first_fraction]"""
import glob
import os
import re
import sqlite3
import sys

path = sys.argv[1]
if os.path.isdir(path):
    path = glob.glob(os.path.join(path, '**', '*results.db'), recursive=True)[0]
skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.2
c = sqlite3.connect(path)
cols = [r[1] for r in c.execute('pragma table_info(kernels)').fetchall()]
cand = [('start', 'end'), ('begin_ns', 'end_ns'), ('start_ns', 'end_ns'), ('begin', 'end')]
found = [x for x in cand if x[0] in cols and x[1] in cols]
if not found:
    sys.exit('no start/end columns in kernels: %s' % cols)
b, e = found[0]
rows = sorted(c.execute('select %s, %s, name from kernels' % (b, e)).fetchall())
t0, t1 = rows[0][0], max(r[1] for r in rows)
t0 = t0 + (t1 - t0) * skip  # steady state: drop the warm-up
rows = [r for r in rows if r[0] >= t0]
busy, cur_s, cur_e = 0, None, None
for s, en, _ in rows:
    if cur_e is None or s > cur_e:
        if cur_e is not None:
            busy += cur_e - cur_s
        cur_s, cur_e = s, en
    else:
        cur_e = max(cur_e, en)
busy += cur_e - cur_s
span = max(r[1] for r in rows) - t0
pnet = [r for r in rows if 'k_pnet' in r[2]]
pb, ps, pe = 0, None, None
for s, en, _ in pnet:
    if pe is None or s > pe:
        if pe is not None:
            pb += pe - ps
        ps, pe = s, en
    else:
        pe = max(pe, en)
if pe is not None:
    pb += pe - ps
print('span %.2f ms, any kernel running %.1f %%, a k_pnet launch running %.1f %%, kernels %d'
      % (span / 1e6, 100 * busy / span, 100 * pb / span, len(rows)))

"""Summarise a rocprofv3 results db (or kernel_stats.csv): per-kernel calls, total, avg (us)."""
import sqlite3, sys, re, glob, os
path = sys.argv[1]
if os.path.isdir(path):
    path = glob.glob(os.path.join(path, '**', '*results.db'), recursive=True)[0]
c = sqlite3.connect(path)
rows = c.execute("select name, count(*), sum(duration), avg(duration), max(vgpr_count), max(accum_vgpr_count), max(sgpr_count), max(lds_size), max(scratch_size) from kernels group by name order by sum(duration) desc").fetchall()
tot = sum(r[2] for r in rows)
print('%-70s %6s %10s %10s %5s %5s %5s %7s %6s' % ('kernel', 'calls', 'total_us', 'avg_us', 'vgpr', 'agpr', 'sgpr', 'lds', 'scr'))
for n, k, s, a, v, ag, sg, l, sc in rows[:int(sys.argv[2]) if len(sys.argv) > 2 else 25]:
    n = re.sub(r'\(anonymous namespace\)::', '', n); n = re.sub(r'\(.*', '', n)[:70]
    print('%-70s %6d %10.1f %10.2f %5s %5s %5s %7s %6s  %4.1f%%' % (n, k, s / 1e3, a / 1e3, v, ag, sg, l, sc, 100 * s / tot))
print('total %.1f us' % (tot / 1e3))

"""Per-launch listing of one det-batch's stage-2/3 (RNet / ONet) kernels from a rocprofv3 db:
python scripts/cand_layers.py DIR"""
import glob, re, sqlite3, sys
p = glob.glob(sys.argv[1] + '/**/*results.db', recursive=True)[0]
rows = sqlite3.connect(p).execute(
    "select name,start,end,duration,grid_x,grid_y,grid_z,workgroup_x from kernels order by start").fetchall()
starts = [i for i, r in enumerate(rows) if 'k_cand_front' in r[0] and '24' in r[0]]
i0 = starts[len(starts) // 2]
i1 = next(i for i in range(i0 + 1, len(rows)) if 'k_pnet' in rows[i][0])
tot = 0
for r in rows[i0:i1]:
    n = re.sub(r'\(.*', '', r[0])[:60]
    tot += r[3]
    print('%-60s %8.1f us  grid %7d x %3d x %2d' % (n, r[3] / 1e3, r[4] // max(1, r[7]), r[5], r[6]))
print('total %.1f us over %d launches' % (tot / 1e3, i1 - i0))

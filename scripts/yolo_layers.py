"""Per-launch listing of one YOLO det-batch from a rocprofv3 results db (kernel trace of bench
--config c3 --lanes 1): the launches between two k_letterbox_s3 dispatches, with grid and time."""
import glob, re, sqlite3, sys
p = sys.argv[1]
if not p.endswith('.db'):
    p = glob.glob(p + '/**/*results.db', recursive=True)[0]
rows = sqlite3.connect(p).execute(
    "select name,start,end,duration,grid_x,workgroup_x,stream_id from kernels order by start").fetchall()
lb = [i for i, r in enumerate(rows) if 'letterbox' in r[0] or 'k_yolo_stem' in r[0]]
i0, i1 = lb[-3], lb[-2]
seq = [r for r in rows[i0:i1] if r[6] == rows[i0][6]]
tot = 0.0
for r in seq:
    n = re.sub(r'\(.*', '', re.sub(r'\(anonymous namespace\)::', '', r[0]))[:48]
    tot += r[3] / 1e3
    print('%-48s %8.1f us  grid %7d' % (n, r[3] / 1e3, r[4] // r[5]))
print('det-batch busy %.1f us, span %.1f us, launches %d' % (tot, (seq[-1][2] - seq[0][1]) / 1e3, len(seq)))

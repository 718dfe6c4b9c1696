"""Per-launch timeline of the FaceNet forwards in a rocprofv3 results db: span/busy of every
forward (k_blob or k_stem_head ... k_l2_normalize) and the per-kernel listing of the largest one."""
import glob, re, sqlite3, sys
p = sys.argv[1]
if not p.endswith('.db'):
    p = glob.glob(p + '/**/*results.db', recursive=True)[0]
rows = sqlite3.connect(p).execute(
    "select name,start,end,duration,grid_x,grid_y,grid_z,workgroup_x,stream_id from kernels order by start").fetchall()
heads = [i for i, r in enumerate(rows) if 'k_l2_normalize' in r[0] or 'k_facenet_head' in r[0]]
fw = []
for h in heads:
    s = h
    while s > 0 and 'k_blob' not in rows[s][0] and 'k_stem_head' not in rows[s][0]:
        s -= 1
    seq = [r for r in rows[s:h + 1] if r[8] == rows[h][8]]
    fw.append((sum(r[3] for r in seq), seq))
print('forwards:', ' '.join('%.0f' % (b / 1e3) for b, _ in fw), 'us busy')
busy, seq = max(fw, key=lambda t: t[0])
agg = {}
for r in seq:
    n = re.sub(r'\(anonymous namespace\)::', '', r[0]); n = re.sub(r'\(.*', '', n).replace('_ZN3vtf6k_convIDF16bLi', 'conv').replace('EEEvNS_10ConvParamsE', '')[:44]
    if len(sys.argv) > 2:
        print('%-44s %8.1f us  grid %6d x %4d x %2d' % (n, r[3] / 1e3, r[4] // r[7], r[5], r[6]))
    a = agg.setdefault(n, [0, 0.0])
    a[0] += 1
    a[1] += r[3] / 1e3
for n, (k, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print('%-44s %4d %9.1f us' % (n, k, t))
print('largest forward: span %.1f us busy %.1f us launches %d' % ((seq[-1][2] - seq[0][1]) / 1e3, busy / 1e3, len(seq)))

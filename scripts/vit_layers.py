"""Per-launch durations of one ViT forward in a rocprofv3 results db: the kernels between a
k_vit_tokens launch and the next k_layernorm<false> (final CLS LayerNorm), grouped by kind and
by GEMM grid (q|k|v, proj, fc1, fc2 have distinct grids)."""
import glob, re, sqlite3, sys
p = sys.argv[1]
if not p.endswith('.db'):
    p = glob.glob(p + '/**/*results.db', recursive=True)[0]
rows = sqlite3.connect(p).execute(
    "select name,duration,grid_x,grid_y,workgroup_x from kernels order by start").fetchall()
starts = [i for i, r in enumerate(rows) if 'k_vit_tokens' in r[0]]
i0 = starts[len(starts) // 2]
agg = {}
for r in rows[i0:]:
    n = re.sub(r'\(anonymous namespace\)::', '', r[0])
    n = re.sub(r'\(.*', '', n)[:48]
    if 'k_layernorm<false>' in n:
        break
    key = '%s grid %d' % (n, r[2] // r[4])
    a = agg.setdefault(key, [0, 0.0])
    a[0] += 1
    a[1] += r[1] / 1e3
tot = sum(v[1] for v in agg.values())
for k, (c, t) in sorted(agg.items(), key=lambda kv: -kv[1][1]):
    print('%-64s %4d x %8.2f us = %9.1f us  %4.1f%%' % (k, c, t / c, t, 100 * t / tot))
print('forward busy %.1f us' % tot)

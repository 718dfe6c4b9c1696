"""Static instruction mix of one kernel in a `-gline-tables-only` device assembly, by source
line range (phase) and basic block.  usage: isa_lines.py file.s mangled-prefix [src.hip]
Phases are given as 'name:first-last' source-line ranges in PHASES (env ISA_PHASES)."""
import collections
import os
import re
import sys

asm, prefix = sys.argv[1], sys.argv[2]
L = open(asm).read().split('\n')
s = next(i for i, l in enumerate(L) if l.startswith(prefix) and l.split(':')[0].startswith(prefix) and ':' in l
         and not l.startswith('\t'))
e = next(i for i in range(s, len(L)) if L[i].startswith('.Lfunc_end'))
phases = [(p.split(':')[0], *map(int, p.split(':')[1].split('-'))) for p in os.environ.get('ISA_PHASES', '').split()]


def kind(op):
    if op.startswith('v_mfma'):
        return 'mfma'
    if op.startswith('v_pk_'):
        return 'vpk'
    if op.startswith('v_'):
        return 'valu'
    if op.startswith('s_'):
        return 'salu'
    if op.startswith('ds_'):
        return 'lds'
    if op.startswith(('buffer', 'global', 'flat')):
        return 'vmem'
    if op.startswith('scratch'):
        return 'scratch'
    return 'other'


line = 0
per = collections.defaultdict(collections.Counter)
blocks = []
cur = None
for l in L[s:e]:
    t = l.strip()
    m = re.match(r'\.loc\s+\d+\s+(\d+)', t)
    if m:
        line = int(m.group(1))
        continue
    if t.endswith(':') and not t.startswith(';'):
        cur = [t[:-1], collections.Counter(), line]
        blocks.append(cur)
        continue
    if not t or t.startswith(('.', ';')):
        continue
    op = t.split()[0]
    k = kind(op)
    ph = next((p[0] for p in phases if p[1] <= line <= p[2]), 'other')
    per[ph][k] += 1
    per[ph]['line:%d' % line] += 0
    if cur:
        cur[1][k] += 1
tot = collections.Counter()
for ph, c in per.items():
    cc = {k: v for k, v in c.items() if not k.startswith('line')}
    tot.update(cc)
    print('%-10s %s' % (ph, dict(sorted(cc.items()))))
print('%-10s %s' % ('total', dict(sorted(tot.items()))))
if os.environ.get('ISA_BLOCKS'):
    for b, c, ln in blocks:
        print(b, ln, dict(c))

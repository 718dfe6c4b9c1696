"""Highest VGPR index referenced per basic block of one kernel in a device .s (a proxy for where
register pressure peaks).  usage: isa_pressure.py file.s mangled-prefix [top]"""
import re
import sys

L = open(sys.argv[1]).read().split('\n')
pre = sys.argv[2]
top = int(sys.argv[3]) if len(sys.argv) > 3 else 15
s = next(i for i, l in enumerate(L) if l.startswith(pre) and not l.startswith('\t') and l.split(':')[0].startswith(pre))
e = next(i for i in range(s, len(L)) if L[i].startswith('.Lfunc_end'))
blocks, cur, line = [], None, 0
for l in L[s:e]:
    t = l.strip()
    m = re.match(r'\.loc\s+0\s+(\d+)', t)
    if m:
        line = int(m.group(1))
        if cur:
            cur['lines'].add(line)
        continue
    if re.match(r'^\.LBB\d+_\d+:', t):
        cur = {'name': t.split(':')[0], 'max': -1, 'n': 0, 'lines': set()}
        blocks.append(cur)
        continue
    if cur is None or not t or t.startswith(('.', ';')):
        continue
    cur['n'] += 1
    if t.startswith(('v_writelane', 'v_readlane', 'scratch_')):
        continue  # SGPR-spill lanes and VGPR spill traffic
    for a, b in re.findall(r'\bv\[(\d+):(\d+)\]', t):
        cur['max'] = max(cur['max'], int(b))
    for a in re.findall(r'\bv(\d+)\b', t):
        cur['max'] = max(cur['max'], int(a))
for b in sorted(blocks, key=lambda b: -b['max'])[:top]:
    ln = sorted(x for x in b['lines'] if x)
    print(b['name'], 'vmax', b['max'], 'instrs', b['n'], 'src', (ln[0], ln[-1]) if ln else '')

#!/bin/bash
# FETCH_SIZE per launch for known byte counts at 16 / 12 / 4 B per lane and the PR window pattern
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6cal_${1:-a}
mkdir -p $O
timeout -k 10 60 ./scripts/calib_fetch > $O/plain.txt 2>&1 || { cat $O/plain.txt; exit 1; }
cat $O/plain.txt
timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/fetch -o run -- ./scripts/calib_fetch > $O/fetch.out 2> $O/fetch.err || { tail -5 $O/fetch.err; exit 1; }
python3 - "$O" <<'EOF'
import csv, glob, os, re, sys
from collections import defaultdict
d = sys.argv[1]
f = glob.glob(os.path.join(d, 'fetch', '**', '*counter_collection.csv'), recursive=True)[0]
per = defaultdict(list)
for r in csv.DictReader(open(f)):
    if r['Counter_Name'] != 'FETCH_SIZE':
        continue
    n = re.sub(r'\(.*', '', r['Kernel_Name']).replace('void ', '')
    per[n].append(float(r['Counter_Value']) * 1024)
B = 3 << 28
win = None
for line in open(os.path.join(d, 'plain.txt')):
    m = re.search(r'window reads (\d+) bytes', line)
    if m:
        win = int(m.group(1))
    m2 = re.search(r'level (\d+) distinct', line)
    if m2:
        lvl = int(m2.group(1))
for n, v in sorted(per.items()):
    ref = B if n != 'tile12' else win
    print('%-8s launches %d  FETCH_SIZE %s MB  / known bytes %.1f MB = %s' % (
        n, len(v), ' '.join('%.1f' % (x / 1e6) for x in v), ref / 1e6, ' '.join('%.3f' % (x / ref) for x in v)))
print('tile12 level bytes %.1f MB: FETCH / level = %s' % (lvl / 1e6, ' '.join('%.3f' % (x / lvl) for x in per['tile12'])))
EOF

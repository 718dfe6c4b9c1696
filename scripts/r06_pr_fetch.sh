#!/bin/bash
# k_pnet FETCH_SIZE per launch (x 2, calibrated for 4/12/16-B loads: profiles/r06_fetch_calibration.txt)
# under phase-skip masks (VTF_PNET_DEBUG; 16 = candidate output off, +1 fill, +2 conv1 (PR: also
# its level reads), +4 conv2, +8 conv3, +32 heads, +64 staging): where the PR launch's bytes come from
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6prf_${1:-a}
MASKS=${2:-"16 18 20 24 48 127"}
mkdir -p $O
for m in $MASKS; do
  VTF_PNET_DEBUG=$m timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/m$m -o run -- python3 scripts/probe_pnet.py child > $O/m$m.txt 2> $O/m$m.err || { tail -5 $O/m$m.err; exit 1; }
  python3 - "$O/m$m" "$m" <<'PY'
import csv, glob, re, sys
from collections import defaultdict
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0]
acc, ids = defaultdict(float), defaultdict(set)
for r in csv.DictReader(open(f)):
    n = r['Kernel_Name']
    if 'k_pnet' not in n and 'resample' not in n:
        continue
    k = re.sub(r'\(.*', '', n).replace('void ', '').replace('vtf::', '')
    acc[k] += float(r['Counter_Value']) * 1024 * 2
    ids[k].add(r.get('Dispatch_Id') or r.get('Correlation_Id'))
print('mask', sys.argv[2], ' | '.join('%s %.1f MB/launch x%d' % (k, acc[k] / len(ids[k]) / 1e6, len(ids[k])) for k in sorted(acc)))
PY
done
find $O -name '*.csv' -size +5M -delete

#!/bin/bash
# k_pnet LDS bank-conflict cycles per phase: SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE per launch under
# phase-skip masks (VTF_PNET_DEBUG: 16 base, +1 fill, +2 conv1 (PR: and its level fill), +4 conv2, +8 conv3, +32 heads)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6ldc_${1:-a}
MASKS=${2:-"16 17 18 20 24 48"}
mkdir -p $O
for m in $MASKS; do
  VTF_PNET_DEBUG=$m timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_IDX_ACTIVE SQ_LDS_BANK_CONFLICT SQ_INSTS_LDS SQ_WAVES --kernel-trace --output-format csv -d $O/m$m -o run -- python3 scripts/probe_pnet.py child > $O/m$m.txt 2> $O/m$m.err || { tail -5 $O/m$m.err; exit 1; }
  python3 - "$O/m$m" "$m" <<'PY'
import csv, glob, re, sys
from collections import defaultdict
f = glob.glob(sys.argv[1] + '/**/*counter_collection.csv', recursive=True)[0]
acc, ids = defaultdict(lambda: defaultdict(float)), defaultdict(set)
for r in csv.DictReader(open(f)):
    n = r['Kernel_Name']
    if 'k_pnet' not in n:
        continue
    k = 'X ' if 'true, false, false' in n else 'PR'
    acc[k][r['Counter_Name']] += float(r['Counter_Value'])
    ids[k].add(r.get('Dispatch_Id') or r.get('Correlation_Id'))
out = []
for k in sorted(acc):
    a, n = acc[k], len(ids[k])
    out.append('%s conflict %.3g active %.3g (%.1f %%) lds-insts/wave %.0f' % (
        k, a['SQ_LDS_BANK_CONFLICT'] / n, a['SQ_LDS_IDX_ACTIVE'] / n, 100 * a['SQ_LDS_BANK_CONFLICT'] / max(1, a['SQ_LDS_IDX_ACTIVE']),
        a['SQ_INSTS_LDS'] / max(1, a['SQ_WAVES'])))
print('mask', sys.argv[2], ' | '.join(out))
PY
done
find $O -name '*.csv' -size +5M -delete

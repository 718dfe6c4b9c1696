#!/bin/bash
# k_resample_sat_multi level rows per workgroup tile (VTF_RS_TH 8 / 16 / 32): MTCNN GPU tests at 32,
# FETCH_SIZE and kernel time per setting (probe_pnet child), c2 300 det-batches 8 vs 32 interleaved
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6rs_${1:-a}
mkdir -p $O
VTF_RS_TH=32 timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for th in 8 16 32; do
  VTF_RS_TH=$th timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/f$th -o run -- python3 scripts/probe_pnet.py child > /dev/null 2> $O/f$th.err || { tail -5 $O/f$th.err; exit 1; }
  VTF_RS_TH=$th timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $O/t$th -o run -- python3 scripts/probe_pnet.py child > /dev/null 2> $O/t$th.err || { tail -5 $O/t$th.err; exit 1; }
  python3 - "$O" "$th" <<'PY'
import csv, glob, sys
from collections import defaultdict
O, th = sys.argv[1], sys.argv[2]
f = glob.glob(O + '/f' + th + '/**/*counter_collection.csv', recursive=True)[0]
acc, ids = 0.0, set()
for r in csv.DictReader(open(f)):
    if 'k_resample_sat_multi' in r['Kernel_Name']:
        acc += float(r['Counter_Value']) * 1024 * 2
        ids.add(r.get('Dispatch_Id') or r.get('Correlation_Id'))
s = glob.glob(O + '/t' + th + '/**/*kernel_stats.csv', recursive=True)[0]
ns = [float(r['AverageNs']) for r in csv.DictReader(open(s)) if 'k_resample_sat_multi' in r['Name']]
print('RS_TH %s: fetch %.1f MB per launch, %.1f us per launch' % (th, acc / max(1, len(ids)) / 1e6, ns[0] / 1e3 if ns else -1))
PY
done
for rep in 1 2; do
  for th in 8 32; do
    VTF_RS_TH=$th timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('RS_TH $th c2', d['value'], d['ms_per_step'], d['faces_per_frame'])"
  done
done
find $O -name '*.csv' -size +5M -delete
find $O -name '*.db' -delete

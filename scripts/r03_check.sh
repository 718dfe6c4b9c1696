#!/bin/bash
# GPU tests + smoke, then the default bench (config 2, 10k frames); logs under gpurun_out/TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r03a}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v -rA --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/tests.log | tail -3
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 500 python3 bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
python3 -c "
import json; r = json.load(open('$O/bench_c2.json'))
print('c2', r['value'], r['unit'], 'ms/step', r['ms_per_step'], 'faces/frame', r['faces_per_frame'], 'roof', r['roofline']['frac'], r['roofline']['avg_launch_ms'], 'sustained', r.get('sustained', {}).get('value'), 'cpu', r['cpu_baseline']['value'])"

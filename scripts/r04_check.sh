#!/bin/bash
# GPU tests (-rA: print() lines of passing tests too) + smoke, then the default bench (config 2,
# 10k frames) and config 5 (distinct device-generated 1080p frames, grouping leg); logs under
# gpurun_out/TAG.  Each GPU step has its own time limit; the script stops at the first failure.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04a}
mkdir -p $O
timeout -k 10 700 python -u -m pytest -v -rA --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/tests.log | tail -3
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
python3 - $O <<'PY'
import json, sys
r = json.load(open(sys.argv[1] + '/bench_c2.json'))
e = r['roofline_e2e']
print('c2', r['value'], 'ms/step', r['ms_per_step'], 'faces/frame', r['faces_per_frame'], 'k_pnet frac', r['roofline']['frac'],
      r['roofline']['avg_launch_ms'], 'e2e frac', e['frac'], 'bound ms', e['bound_ms_per_step'], 'cpu', r['cpu_baseline']['value'])
PY
if [ "${2:-}" = c5 ]; then
  timeout -k 10 400 python3 bench.py --config c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
  python3 - $O <<'PY'
import json, sys
r = json.load(open(sys.argv[1] + '/bench_c5.json'))
print('c5', r['value'], 'ms/step', r['ms_per_step'], 'e2e', r['roofline_e2e']['frac'], 'grouping', r['grouping'])
PY
fi

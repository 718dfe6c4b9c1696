#!/bin/bash
# Round-6 check on one box: GPU tests (optionally a -k filter), smoke, the driver-shaped bench line.
# bash scripts/r06_check.sh TAG ["pytest -k expr"] [bench args...]
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6_${1:-a}
K=${2:-}
shift 2 2>/dev/null
mkdir -p $O
if [ -n "$K" ]; then
  timeout -k 10 900 python -u -m pytest -v -rA --timeout 300 --timeout-method thread -m gpu tests -k "$K" > $O/tests.log 2>&1
else
  timeout -k 10 900 python -u -m pytest -v -rA --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
fi
rc=$?
grep -E "passed|failed|error" $O/tests.log | tail -3
grep -E "^FAILED|^ERROR" $O/tests.log | head -20
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
tail -1 $O/smoke.log
timeout -k 10 900 python3 bench.py "$@" > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "
import json; r = json.load(open('$O/bench.json'))
print('bench', r['value'], r['unit'], 'ms/step', r['ms_per_step'], 'faces/frame', r.get('faces_per_frame'), 'roof', r['roofline']['frac'], r['roofline']['avg_launch_ms'], 'sustained', r.get('sustained', {}).get('value'), 'cpu', (r.get('cpu_baseline') or {}).get('value'), (r.get('cpu_baseline') or {}).get('sample'))"

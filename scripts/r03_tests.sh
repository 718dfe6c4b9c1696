#!/bin/bash
# GPU test suite (one process) + smoke; logs under gpurun_out/t_TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/t_${1:-a}
shift
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v -rA --timeout 300 --timeout-method thread -m gpu "${@:-tests}" > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/tests.log | tail -3
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log

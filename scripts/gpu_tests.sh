#!/bin/bash
# full GPU test suite (one process) + smoke; logs under gpurun_out/gt_TAG
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/gt_${1:-a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1 || true
grep -E "passed|failed|error" $O/tests.log | tail -3
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1
tail -1 $O/smoke.log

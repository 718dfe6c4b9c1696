#!/bin/bash
# The .y4m frame source on one box: its tests, scripts/bench_y4m.py (kernel + read() rate) and a
# kernel trace of the same.  bash scripts/r05_y4m.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/y4m_${1:-a}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v --timeout 200 --timeout-method thread tests/test_video.py > $O/tests.log 2>&1 || exit $?
tail -1 $O/tests.log
timeout -k 10 120 python3 scripts/bench_y4m.py $O/bench_y4m.json > $O/bench.log 2>&1 || exit $?
cat $O/bench.log
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 scripts/bench_y4m.py > $O/prof.log 2>&1 || exit $?
python3 scripts/kstats.py $O/prof 10 > $O/kernel_stats.txt 2>&1
find $O -name '*.db' -delete
cat $O/kernel_stats.txt

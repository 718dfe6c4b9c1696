#!/bin/bash
# FaceNet fused-block check: parity tests, interleaved timing, one-lane kernel stats
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04fn}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -v -rA --timeout 200 --timeout-method thread -m gpu tests/test_facenet_gpu.py > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error|fused vs" $O/tests.log | tail -5
[ $rc -le 1 ] || exit $rc
timeout -k 10 200 python3 scripts/facenet_time.py 20 > $O/time.log 2>&1 || exit $?
cat $O/time.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/raw -o run -- python3 scripts/facenet_time.py 3 1 > $O/prof.log 2>&1 || exit $?
python3 scripts/kstats.py $O/raw 40 > $O/kernel_stats.txt 2>&1
rm -rf $O/raw
head -20 $O/kernel_stats.txt

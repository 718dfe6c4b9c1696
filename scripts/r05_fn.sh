#!/bin/bash
# FaceNet: identity tests, forward timing A/B of Block17 split vs fused vs unfused, kernel stats
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05fn}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v -s --timeout 300 --timeout-method thread -m gpu tests/test_facenet_gpu.py > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error|FAILED|fused vs" $O/tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/facenet_time.py 20 "VTF_B17_SPLIT=1,VTF_B17_SPLIT=0,0" > $O/time.txt 2>&1 || exit $?
cat $O/time.txt
VTF_B17_SPLIT=1 timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/raw -o run -- python3 scripts/facenet_time.py 5 "VTF_B17_SPLIT=1" > /dev/null 2>&1 || exit $?
python3 scripts/kstats.py $O/raw 30 > $O/kernel_stats.txt 2>&1
rm -rf $O/raw
head -25 $O/kernel_stats.txt

#!/bin/bash
# NMS timing (scripts/nms_time.py) plain and under the kernel tracer
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04nms}
mkdir -p $O
timeout -k 10 200 python3 scripts/nms_time.py 20 > $O/time.log 2>&1 || exit $?
cat $O/time.log
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/raw -o run -- python3 scripts/nms_time.py 10 > $O/prof.log 2>&1 || exit $?
python3 scripts/kstats.py $O/raw 25 > $O/kernel_stats.txt 2>&1
rm -rf $O/raw
head -25 $O/kernel_stats.txt

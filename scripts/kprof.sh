#!/bin/bash
# one-lane kernel trace of a bench config, summarised on the box: bash scripts/kprof.sh TAG CONFIG [bench args]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; CFG=$2; shift 2
O=gpurun_out/kp_$TAG
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/raw -o run -- python3 bench.py --config $CFG --steps 10 --warmup 3 --no-cpu-baseline --no-extras --sustain-frames 0 "$@" > $O/bench.json 2> $O/err.txt
rc=$?
python3 scripts/kstats.py $O/raw 40 > $O/kernel_stats.txt 2>&1
rm -rf $O/raw
exit $rc

#!/bin/bash
# HIP hardware queues per process (GPU_MAX_HW_QUEUES, default 4) x lanes, c2, interleaved
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/hwq_${1:-a}
mkdir -p $O
for rep in 1 2; do
  for cfg in "4 3" "8 3" "8 4" "8 5"; do
    set -- $cfg
    GPU_MAX_HW_QUEUES=$1 timeout -k 10 300 python3 bench.py --steps 300 --lanes $2 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('hwq=$1 lanes=$2 c2', d['value'], d['ms_per_step'])"
  done
done

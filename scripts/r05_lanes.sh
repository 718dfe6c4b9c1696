#!/bin/bash
# c2 throughput by lane count (and 8 HW queues at 4 lanes), this build, interleaved
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05ln}
mkdir -p $O
for rep in 1 2; do
  for v in 3 2 4 4q 5q; do
    case $v in 4q) L=4; E="GPU_MAX_HW_QUEUES=8";; 5q) L=5; E="GPU_MAX_HW_QUEUES=8";; *) L=$v; E="";; esac
    env $E timeout -k 10 300 python3 bench.py --steps 300 --lanes $L --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('lanes $v', 'c2', d['value'], d['ms_per_step'])"
  done
done

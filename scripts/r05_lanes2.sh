#!/bin/bash
# lanes x HW queues on one box, interleaved: bash scripts/r05_lanes2.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05ln3}
mkdir -p $O
B="--steps 300 --no-cpu-baseline --no-extras --sustain-frames 0"
for rep in 1 2; do
  for lq in "4 8" "5 10" "6 12" "4 16"; do
    set -- $lq
    timeout -k 10 300 python3 bench.py --lanes $1 --hw-queues $2 $B > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('lanes $1 queues $2 c2', d['value'], d['ms_per_step'])"
  done
done

#!/bin/bash
# lane start-up stagger on 20-det-batch windows: none / after the previous lane's first det-batch
# / 2 ms / 4 ms per lane, interleaved
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6stg_${1:-a}
mkdir -p $O
for rep in 1 2 3 4; do
  for m in "0 0" "1 0" "0 2" "0 4"; do
    set -- $m
    VTF_LANE_STAGGER=$1 VTF_LANE_STAGGER_MS=$2 timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('stagger event $1 ms $2: c2 20', d['value'], d['ms_per_step'])"
  done
done
for m in "0 0" "1 0"; do
  set -- $m
  VTF_LANE_STAGGER=$1 VTF_LANE_STAGGER_MS=$2 timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-extras --sustain-frames 10000 > $O/c2.json 2> $O/c2.err || exit $?
  python3 -c "import json; d=json.load(open('$O/c2.json')); print('stagger event $1 ms $2: c2 625', d['value'], d['ms_per_step'])"
done

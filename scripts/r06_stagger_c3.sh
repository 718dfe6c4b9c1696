#!/bin/bash
# lane start stagger for config 3 (YOLO det-batch 32) and c2 fine steps: 20-det-batch windows
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6stg3_${1:-a}
mkdir -p $O
for rep in 1 2 3; do
  for ms in 0 5 10; do
    VTF_LANE_STAGGER_MS=$ms timeout -k 10 300 python3 bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --no-extras > $O/c3.json 2> $O/c3.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c3.json')); print('c3 stagger ms $ms: 20', d['value'], d['ms_per_step'])"
  done
done
for rep in 1 2 3; do
  for ms in 1 2 3; do
    VTF_LANE_STAGGER_MS=$ms timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('c2 stagger ms $ms: 20', d['value'], d['ms_per_step'])"
  done
done

#!/bin/bash
# arena growth factor (VTF_ARENA_GROW halves: 3 = 1.5x default, 8 = 4x) on 20-det-batch c2 windows
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6ar_${1:-a}
mkdir -p $O
for rep in 1 2 3 4 5; do
  for g in 3 8; do
    VTF_ARENA_GROW=$g timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('grow $g c2 20', d['value'], d['ms_per_step'])"
  done
done

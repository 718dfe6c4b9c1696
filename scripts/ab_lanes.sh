#!/bin/bash
# headline A/B over --lanes (c2, 200 det-batches per run, no extras), interleaved twice
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/lanes
for rep in 1 2; do
  for L in ${1:-2 3 4}; do
    timeout -k 10 200 python3 bench.py --steps 200 --warmup 4 --lanes $L --no-cpu-baseline --no-extras > gpurun_out/lanes/l$L.json 2> gpurun_out/lanes/l$L.err
    python3 -c "import json; d=json.load(open('gpurun_out/lanes/l$L.json')); print('lanes $L rep $rep', d['value'], d['ms_per_step'])"
  done
done

#!/bin/bash
# with the k_pnet quota: quota 1 / 2 / 4 at 3 lanes, then lanes 3 / 4 at the default quota
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ql_${1:-a}
mkdir -p $O
for rep in 1 2; do
  for q in 1 2 4; do
    VTF_PNET_QUOTA=$q timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('quota=$q c2', d['value'], d['ms_per_step'])"
  done
done
for rep in 1 2; do
  for L in 3 4; do
    timeout -k 10 300 python3 bench.py --steps 300 --lanes $L --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('lanes=$L c2', d['value'], d['ms_per_step'])"
  done
done

#!/bin/bash
# c2 3-lane A/B: exact k_pnet at 4 vs 3 workgroups per CU, then lanes 2 / 3 / 4 (default wg)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/xwl_${1:-a}
mkdir -p $O
for rep in 1 2; do
  for wg in 4 3; do
    VTF_PNET_X_WG_PER_CU=$wg timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('xwg=$wg c2', d['value'], d['ms_per_step'])"
  done
done
for rep in 1 2; do
  for L in 2 3 4; do
    timeout -k 10 300 python3 bench.py --steps 300 --lanes $L --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('lanes=$L c2', d['value'], d['ms_per_step'])"
  done
done

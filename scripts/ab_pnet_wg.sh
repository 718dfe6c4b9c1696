#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pw_${1:-a}
mkdir -p $O
for rep in 1 2; do
for w in 3 2; do
  VTF_PNET_WG_PER_CU=$w timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err
  python3 -c "import json; d=json.load(open('$O/c2.json')); print('c2 pnet_wg=$w', d['value'], d['ms_per_step'])"
done
done

#!/bin/bash
# k_pnet chunk x quota (tiles per workgroup) on the default c2 run (625 det-batches), interleaved
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6kn_${1:-a}
mkdir -p $O
for rep in 1 2; do
  for cfg in "4 2" "4 1" "4 4" "2 4" "8 1" "4 3"; do
    set -- $cfg
    VTF_PNET_CHUNK=$1 VTF_PNET_QUOTA=$2 timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-extras --sustain-frames 10000 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('chunk $1 quota $2 c2 625', d['value'], d['ms_per_step'])"
  done
done

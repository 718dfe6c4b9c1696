#!/bin/bash
# k_pnet tiles per chunk (VTF_PNET_CHUNK) re-checked after the PR fill fix: c2 300 det-batches, interleaved
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6chk_${1:-a}
mkdir -p $O
for rep in 1 2; do
  for c in 4 2 8; do
    VTF_PNET_CHUNK=$c timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('chunk $c c2', d['value'], d['ms_per_step'], d['faces_per_frame'])"
  done
done

#!/bin/bash
# FaceNet Block17 stage 4 per image (VTF_B17_SPLIT=0) vs the batch tail launch, on c2 (625 det-batches)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6b17c2_${1:-a}
mkdir -p $O
for rep in 1 2 3; do
  for v in 1 0; do
    VTF_B17_SPLIT=$v timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-extras --sustain-frames 10000 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('b17 split $v c2 625', d['value'], d['ms_per_step'])"
  done
done

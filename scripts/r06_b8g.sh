#!/bin/bash
# FaceNet Block8 middle images per workgroup (VTF_B8_G 1 / 3 / 7): solo forward and c2 625, interleaved
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6b8_${1:-a}
mkdir -p $O
for g in 1 3 7; do
  VTF_B8_G=$g timeout -k 10 200 python3 -u scripts/r06_b17ws.py 20 "VTF_B8_G=$g" facenet > $O/fn$g.txt 2> $O/fn$g.err || exit $?
  echo "b8 g $g $(grep forward $O/fn$g.txt)"
done
for rep in 1 2; do
  for g in 1 3 7; do
    VTF_B8_G=$g timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-extras --sustain-frames 10000 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('b8 g $g c2 625', d['value'], d['ms_per_step'])"
  done
done

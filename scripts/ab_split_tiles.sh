#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/st_${1:-a}
mkdir -p $O
for t in 64 129; do
VTF_DMA_SPLIT64=$t timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mtcnn_gpu.py > $O/tests_$t.log 2>&1
tail -1 $O/tests_$t.log
done
for rep in 1 2; do
for t in 128 64 129; do
  VTF_DMA_SPLIT64=$t timeout -k 10 300 python3 bench.py --steps 200 --no-cpu-baseline --no-extras --sustain-frames 0 --lanes 1 > $O/c2.json 2> $O/c2.err
  python3 -c "import json; d=json.load(open('$O/c2.json')); print('c2 1-lane tile=$t', d['value'], d['ms_per_step'])"
done
done

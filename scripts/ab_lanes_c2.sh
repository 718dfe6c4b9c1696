#!/bin/bash
# c2 3-lane bench, interleaved repeats (tag) + under-tracer kernel stats with 3 lanes
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/l3_${1:-a}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mtcnn_gpu.py > $O/tests.log 2>&1
tail -1 $O/tests.log
for rep in 1 2 3; do
  timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err
  python3 -c "import json; d=json.load(open('$O/c2.json')); print('c2', d['value'], d['ms_per_step'])"
done

#!/bin/bash
# span-mode candidate convs: MTCNN GPU tests, c2 3-lane A/B (interleaved, span on / off),
# 1-lane kernel stats with the span kernel
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/span_${1:-a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py > $O/tests.log 2>&1
tail -1 $O/tests.log
for rep in 1 2; do
  for sp in 1 0; do
    VTF_CONV_SPAN=$sp timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2_$sp.json 2> $O/c2_$sp.err
    python3 -c "import json; d=json.load(open('$O/c2_$sp.json')); print('span', $sp, d['value'], d['ms_per_step'])"
  done
done
bash scripts/kprof.sh span_${1:-a} c2 --lanes 1
grep -E "span|conv_dma<1" gpurun_out/kp_span_${1:-a}/kernel_stats.txt

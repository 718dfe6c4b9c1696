#!/bin/bash
# span-pool B stages A/B (VTF_SPOOL_NS = 2 / 3 / 4): MTCNN tests at 4, 1-lane kernel time, c2 bench
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/sns_${1:-a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py > $O/tests.log 2>&1
tail -1 $O/tests.log
for ns in 2 3 4; do
  VTF_SPOOL_NS=$ns bash scripts/kprof.sh sns$ns c2 --lanes 1
  echo "ns=$ns $(grep 'span_pool' gpurun_out/kp_sns$ns/kernel_stats.txt)"
done
for rep in 1 2; do
  for ns in 2 4; do
    VTF_SPOOL_NS=$ns timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('ns=$ns', 'c2', d['value'], d['ms_per_step'])"
  done
done

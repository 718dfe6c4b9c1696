#!/bin/bash
# exact-levels k_pnet variant A/B (VTF_PNET_X = 1 / 0): MTCNN GPU tests under both, k_pnet solo
# (both launches, events on its stream), c2 3-lane bench interleaved, 1-lane kernel stats
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/px_${1:-a}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py > $O/tests.log 2>&1
tail -1 $O/tests.log
for rep in 1 2; do
  for x in 1 0; do
    VTF_PNET_X=$x timeout -k 10 120 python3 -u scripts/probe_pnet.py child > $O/pnet.txt 2> $O/pnet.err
    echo "X=$x pnet $(tail -1 $O/pnet.txt)"
  done
done
for rep in 1 2; do
  for x in 1 0; do
    VTF_PNET_X=$x timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('X=$x c2', d['value'], d['ms_per_step'])"
  done
done
bash scripts/kprof.sh px_${1:-a} c2 --lanes 1
grep -E "k_pnet" gpurun_out/kp_px_${1:-a}/kernel_stats.txt | cut -c1-160

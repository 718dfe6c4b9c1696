#!/bin/bash
# RNet/ONet on the LDS-DMA split mode: MTCNN GPU tests, c2 A/B (VTF_MTCNN_SP=1/0), 1-lane kernel stats
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ms_${1:-a}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py tests/test_facenet_gpu.py -k "not config5" > $O/tests.log 2>&1
grep -E "passed|failed|error" $O/tests.log | tail -2
for arm in 1 0 1 0; do
  VTF_MTCNN_SP=$arm timeout -k 10 300 python3 bench.py --steps 200 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2_$arm.json 2> $O/c2_$arm.err
  python3 -c "import json; d=json.load(open('$O/c2_$arm.json')); print('c2 sp=$arm', d['value'], d['ms_per_step'])"
done
bash scripts/kprof.sh ms_${1:-a}_k c2 --lanes 1
head -24 gpurun_out/kp_ms_${1:-a}_k/kernel_stats.txt

#!/bin/bash
# k_pnet workgroup quota A/B (VTF_PNET_QUOTA = 0 persistent / 8 / 32 chunks): MTCNN tests with a
# quota, c2 3-lane bench interleaved
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/quota_${1:-a}
mkdir -p $O
VTF_PNET_QUOTA=8 timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py > $O/tests.log 2>&1
echo "quota 8 tests: $(tail -1 $O/tests.log)"
for rep in 1 2; do
  for q in ${QS:-0 8 32}; do
    VTF_PNET_QUOTA=$q timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('quota=$q c2', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done

#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/yx_${1:-a}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_yolo_gpu.py tests/test_shapes_gpu.py -k "yolo or net or detect or letterbox or postprocess" > $O/tests.log 2>&1 || { grep -E "FAIL|Error|error" $O/tests.log | head -20; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
grep -E "map. max err" $O/tests.log | head -6
for arm in x3 fp32; do
  timeout -k 10 400 python3 bench.py --config c3 --det-precision $arm --steps 40 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c3_$arm.json 2> $O/c3_$arm.err
  python3 -c "import json; d=json.load(open('$O/c3_$arm.json')); print('c3 $arm', d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['achieved'])"
done

#!/bin/bash
# YOLO stem head (letterbox + first conv fused): YOLO GPU tests (incl. the bit-identity test),
# the config-3 / config-5 shape tests, then c3 and c5 A/B (VTF_YOLO_STEM=0 / 1) on one box
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05ys}
mkdir -p $O
timeout -k 10 600 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_yolo_gpu.py tests/test_shapes_gpu.py -k "yolo or x3 or stem or config3 or config5 or c3 or chain" > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; grep "stem head" $O/tests.log | head -4; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for v in 0 1; do
    VTF_YOLO_STEM=$v timeout -k 10 300 python3 bench.py --config c3 --steps 40 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c3.json 2> $O/c3.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c3.json')); print('VTF_YOLO_STEM=$v', 'c3', d['value'], d['ms_per_step'], 'roof', d['roofline']['frac'])"
  done
done
for v in 0 1; do
  VTF_YOLO_STEM=$v timeout -k 10 400 python3 bench.py --config c5 --steps 20 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c5.json 2> $O/c5.err || exit $?
  python3 -c "import json; d=json.load(open('$O/c5.json')); print('VTF_YOLO_STEM=$v', 'c5', d['value'], d['ms_per_step'], 'roof', d['roofline']['frac'])"
done

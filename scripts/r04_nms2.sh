#!/bin/bash
# NMS change check: MTCNN + shape GPU tests, NMS timing, then the default bench (c2)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04nms2}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -v -rA --timeout 300 --timeout-method thread -m gpu tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py tests/test_rcnn_gpu.py tests/test_yolo_gpu.py > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/nms_time.py 20 > $O/time.log 2>&1 || exit $?
grep "^n " $O/time.log
timeout -k 10 400 python3 bench.py --no-cpu-baseline > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
python3 -c "
import json; r = json.load(open('$O/bench_c2.json')); print('c2', r['value'], 'ms/step', r['ms_per_step'], 'frac', r['roofline']['frac'])"

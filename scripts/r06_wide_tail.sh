#!/bin/bash
# bf16x3 wide last-round K split (VTF_DMA3_WIDE_TAIL): YOLO GPU tests, c3 A/B interleaved, one-lane layer listing
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6wt_${1:-a}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests/test_yolo_gpu.py \
  "tests/test_shapes_gpu.py::test_config3_det_batch32" "tests/test_shapes_gpu.py::test_config5_chain" > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
for r in 1 2 3; do
  for v in 0 1; do
    VTF_DMA3_WIDE_TAIL=$v timeout -k 10 200 python3 bench.py --config c3 --steps 150 --warmup 3 --no-cpu-baseline --no-extras > $O/c3_${v}_$r.json 2> $O/c3_${v}_$r.err || { tail -5 $O/c3_${v}_$r.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$O/c3_${v}_$r.json')); print('wide_tail $v run $r c3', d['value'], d['ms_per_step'], d['faces_per_frame'], (d.get('roofline') or {}).get('frac'))"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t -o run -- python3 bench.py --config c3 --steps 6 --warmup 2 --lanes 1 --no-cpu-baseline --no-extras > $O/b.json 2> $O/b.err || exit $?
python3 scripts/yolo_layers.py $O/t > $O/layers.txt 2>&1
rm -rf $O/t
grep -E "grid +(840|836|1808|2520|2624)" $O/layers.txt | head -12

#!/bin/bash
# bf16x3 YOLO conv tiles A/B (VTF_DMA3_NW8 = 1: 128 x 128 eight-wave tiles above 64 channels):
# YOLO tests with the switch, 1-lane kernel stats, c3 bench interleaved
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/nw8_${1:-a}
mkdir -p $O
VTF_DMA3_NW8=1 timeout -k 10 500 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_yolo_gpu.py tests/test_shapes_gpu.py -k "yolo or chain" > $O/tests.log 2>&1
echo "nw8 tests: $(tail -1 $O/tests.log)"
for v in 0 1; do
  VTF_DMA3_NW8=$v bash scripts/kprof.sh nw8_$v c3 --lanes 1
  grep -E "k_conv_dma3" gpurun_out/kp_nw8_$v/kernel_stats.txt | sed "s/^/nw8=$v /" | cut -c1-130
done
for rep in 1 2; do
  for v in 0 1; do
    VTF_DMA3_NW8=$v timeout -k 10 400 python3 bench.py --config c3 --no-cpu-baseline --no-extras > $O/c3.json 2> $O/c3.err
    python3 -c "import json; d=json.load(open('$O/c3.json')); print('nw8=$v c3', d['value'], d['ms_per_step'])"
  done
done

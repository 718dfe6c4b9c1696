#!/bin/bash
# k_conv_dma3 (YOLO bf16x3) stage / tile variants (VTF_DMA3): YOLO GPU tests per variant, then c3
# interleaved A/B on one box
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05d3}
shift
VARS=${@:-"0 1 2"}
mkdir -p $O
for v in $VARS; do
  VTF_DMA3=$v timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_yolo_gpu.py > $O/tests_$v.log 2>&1
  rc=$?; echo "variant $v: $(tail -1 $O/tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for v in $VARS; do
    VTF_DMA3=$v timeout -k 10 300 python3 bench.py --config c3 --steps 40 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c3.json 2> $O/c3.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c3.json')); print('VTF_DMA3=$v', 'c3', d['value'], d['ms_per_step'], 'roof', d['roofline']['frac'])"
  done
done

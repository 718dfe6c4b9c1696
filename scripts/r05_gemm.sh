#!/bin/bash
# k_gemm_x3 stage / tile variants (VTF_GEMM_BIG): split-GEMM + ViT GPU tests per variant, then
# c4 (ViT-L, enc-batch 128) interleaved A/B on one box
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05gm}
shift
VARS=${@:-"0 2 3 4"}
mkdir -p $O
for v in $VARS; do
  VTF_GEMM_BIG=$v timeout -k 10 300 python3 -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests/test_gemm_split_gpu.py tests/test_vit_gpu.py > $O/tests_$v.log 2>&1
  rc=$?; echo "variant $v: $(tail -1 $O/tests_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
for rep in 1 2; do
  for v in $VARS; do
    VTF_GEMM_BIG=$v timeout -k 10 300 python3 bench.py --config c4 --steps 30 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c4.json 2> $O/c4.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c4.json')); print('VTF_GEMM_BIG=$v', 'c4', d['value'], d['ms_per_step'], 'roof', d['roofline']['frac'])"
  done
done

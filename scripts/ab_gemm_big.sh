#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/gb_${1:-a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_split_gpu.py tests/test_vit_gpu.py tests/test_shapes_gpu.py -k "gemm or vit" > $O/tests.log 2>&1
grep -E "passed|failed|error" $O/tests.log | tail -2
for arm in 1 0 1 0; do
  VTF_GEMM_BIG=$arm timeout -k 10 300 python3 bench.py --config c4 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c4_$arm.json 2> $O/c4_$arm.err
  python3 -c "import json; d=json.load(open('$O/c4_$arm.json')); print('big=$arm', d['value'], d['ms_per_step'])"
done
bash scripts/vit_prof.sh ${1:-a}

#!/bin/bash
# GEMM tail split-K: parity tests, then ViT-L c4 with / without the tail slices
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/gt2_${1:-a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_split_gpu.py tests/test_vit_gpu.py tests/test_shapes_gpu.py -k "gemm or vit" > $O/tests.log 2>&1
grep -E "passed|failed|error" $O/tests.log | tail -2
for arm in 1 0 1 0; do
  VTF_GEMM_TAIL=$arm timeout -k 10 300 python3 bench.py --config c4 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c4_$arm.json 2> $O/c4_$arm.err
  python3 -c "import json; d=json.load(open('$O/c4_$arm.json')); print('tail=$arm', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --config c4 --no-cpu-baseline --no-extras --steps 20 --sustain-frames 0 > $O/c4_prof.json 2> $O/c4_prof.err
python3 scripts/kstats.py $O/prof 30 > $O/c4_kernel_stats.txt 2>&1 && rm -rf $O/prof
head -8 $O/c4_kernel_stats.txt

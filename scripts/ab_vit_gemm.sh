#!/bin/bash
# pre-split GEMM: parity tests, then ViT-L c4 bench (new vs k_conv staging-split) + kernel stats
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/vg_${1:-a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread tests/test_gemm_split_gpu.py tests/test_vit_gpu.py ${TESTS_EXTRA} > $O/tests.log 2>&1
grep -E "passed|failed|error" $O/tests.log | tail -2
timeout -k 10 300 python3 bench.py --config c4 --no-cpu-baseline --no-extras > $O/c4_new.json 2> $O/c4_new.err
VTF_VIT_GEMM=conv timeout -k 10 300 python3 bench.py --config c4 --no-cpu-baseline --no-extras > $O/c4_conv.json 2> $O/c4_conv.err
python3 -c "
import json
for t in ('new','conv'):
    d=json.load(open('$O/c4_'+t+'.json')); print(t, d['value'], d['ms_per_step'])"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --config c4 --no-cpu-baseline --no-extras --steps 20 --sustain-frames 0 > $O/c4_prof.json 2> $O/c4_prof.err
python3 scripts/kstats.py $O/prof 30 > $O/c4_kernel_stats.txt 2>&1 && rm -rf $O/prof
head -12 $O/c4_kernel_stats.txt

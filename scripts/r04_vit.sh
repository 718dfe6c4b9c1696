#!/bin/bash
# ViT GPU tests, then the config-4 bench line and its kernel trace; logs under gpurun_out/TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04vit}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -v -rA --timeout 200 --timeout-method thread -m gpu tests/test_vit_gpu.py tests/test_gemm_split_gpu.py > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error|max abs" $O/tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 bench.py --config c4 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || exit $?
python3 -c "
import json; r = json.load(open('$O/bench_c4.json'))
print('c4', r['value'], 'ms/step', r['ms_per_step'], 'roof', r['roofline']['frac'], 'e2e', r['roofline_e2e']['frac'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/raw -o run -- python3 bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline > $O/c4_trace.json 2> $O/c4_trace.err || exit $?
python3 scripts/kstats.py $O/raw 20 > $O/c4_kernel_stats.txt 2>&1
rm -rf $O/raw
head -8 $O/c4_kernel_stats.txt

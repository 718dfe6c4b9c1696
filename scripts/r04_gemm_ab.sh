#!/bin/bash
# k_gemm_x3 tile / stage variants (VTF_GEMM_BIG: 0 = 128x128 two stages, 1 = 256x128 two stages,
# 3 = 256x128 three stages, counted vmcnt): GEMM tests under the variant, then interleaved c4 runs
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04gemm}
V=${2:-3}
mkdir -p $O
VTF_GEMM_BIG=$V timeout -k 10 300 python -u -m pytest -v -rA --timeout 200 --timeout-method thread -m gpu tests/test_gemm_split_gpu.py > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error|max" $O/tests.log | tail -10
[ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  for v in 0 $V; do
    VTF_GEMM_BIG=$v timeout -k 10 300 python3 bench.py --config c4 --no-cpu-baseline > $O/c4_${v}_$r.json 2> $O/c4_${v}_$r.err || exit $?
    python3 -c "
import json; r = json.load(open('$O/c4_${v}_$r.json')); print('VTF_GEMM_BIG=$v', r['value'], 'ms/step', r['ms_per_step'], 'roof', r['roofline']['frac'], r['roofline'].get('avg_launch_ms'))"
  done
done

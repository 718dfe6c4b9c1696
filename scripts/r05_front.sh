#!/bin/bash
# wave-per-candidate RNet front: MTCNN / shape GPU tests, one-lane c2 trace, c2 A/B vs the workgroup front
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05fr}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error|FAILED" $O/tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
bash scripts/r04_c2trace.sh ${1:-r05fr}/tr > /dev/null || exit $?
grep -E "cand_front|k_pnet|resample" $O/tr/c2_kernel_stats_1lane.txt
for rep in 1 2; do
  for v in wg wave; do
    [ $v = wg ] && E="VTF_FRONT_WAVE=0" || E="VTF_FRONT_WAVE=1"
    env $E timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$v', 'c2', d['value'], d['ms_per_step'])"
  done
done

#!/bin/bash
# SAT column pass in 256-thread workgroups (VTF_SAT_COLS8=1): MTCNN tests with it, then c2 A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6satc_${1:-a}
mkdir -p $O
VTF_SAT_COLS8=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py -k "mtcnn or sat or detect" > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/tests.log | tail -2; grep -E "^FAILED" $O/tests.log | head
[ $rc -eq 0 ] || exit $rc
for rep in 1 2 3 4 5 6; do
  for v in 0 1; do
    VTF_SAT_COLS8=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('cols8 $v c2 20', d['value'], d['ms_per_step'])"
  done
done
for rep in 1 2; do
  for v in 0 1; do
    VTF_SAT_COLS8=$v timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-extras --sustain-frames 10000 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('cols8 $v c2 625', d['value'], d['ms_per_step'])"
  done
done
VTF_SAT_COLS8=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t1 -o run -- python3 bench.py --steps 32 --warmup 3 --lanes 1 --no-cpu-baseline --no-extras > $O/t1.json 2> $O/t1.err || exit $?
python3 scripts/kstats.py $O/t1 80 | grep -E "k_sat" 
find $O -name '*.db' -delete

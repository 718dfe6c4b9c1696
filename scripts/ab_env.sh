#!/bin/bash
# A/B of one env switch on one box: GPU tests, then c2 3-lane bench with VAR=1 / VAR=0 interleaved,
# then the 1-lane kernel stats (default):  bash scripts/ab_env.sh TAG VAR [tests]
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; VAR=$2
TESTS=${3:-"tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py"}
O=gpurun_out/abe_$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread $TESTS > $O/tests.log 2>&1
tail -1 $O/tests.log
for rep in 1 2; do
  for v in 1 0; do
    env $VAR=$v timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$VAR=$v', 'c2', d['value'], d['ms_per_step'])"
  done
done
bash scripts/kprof.sh $TAG c2 --lanes 1
head -14 gpurun_out/kp_$TAG/kernel_stats.txt

#!/bin/bash
# FaceNet encoder-only + c2 A/B over values of one env switch:  bash scripts/ab_fn_env.sh TAG VAR v1 v2
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; VAR=$2; shift 2
O=gpurun_out/abf_$TAG
mkdir -p $O
for v in "$@"; do
  env $VAR=$v timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_facenet_gpu.py > $O/tests_$v.log 2>&1
  echo "$VAR=$v $(tail -1 $O/tests_$v.log)"
done
for rep in 1 2; do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 300 python3 bench.py --det-model none --enc-model facenet --steps 40 --no-cpu-baseline --no-extras > $O/fn.json 2> $O/fn.err
    python3 -c "import json; d=json.load(open('$O/fn.json')); print('$VAR=$v facenet', d['value'], d['ms_per_step'])"
  done
done
for rep in 1 2; do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$VAR=$v c2', d['value'], d['ms_per_step'])"
  done
done

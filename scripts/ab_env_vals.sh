#!/bin/bash
# c2 3-lane A/B over values of one env switch, interleaved twice:  bash scripts/ab_env_vals.sh TAG VAR v1 v2 ...
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; VAR=$2; shift 2
O=gpurun_out/abv_$TAG
mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$VAR=$v c2', d['value'], d['ms_per_step'])"
  done
done

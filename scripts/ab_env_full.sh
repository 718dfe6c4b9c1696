#!/bin/bash
# full default bench (625 det-batches, no extras) over values of one env switch, interleaved twice
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; VAR=$2; shift 2
O=gpurun_out/abf_$TAG
mkdir -p $O
for rep in 1 2; do
  for v in "$@"; do
    env $VAR=$v timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-extras > $O/c2.json 2> $O/c2.err
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$VAR=$v c2', d['value'], d['ms_per_step'])"
  done
done

#!/bin/bash
# c2 (default lanes) over several environment settings, interleaved twice on one box:
#   bash scripts/r05_envs_ab.sh TAG "A=1" "B=2 C=3" ...   ("-" = the defaults)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=$1; shift
O=gpurun_out/abe_$TAG
mkdir -p $O
for rep in 1 2; do
  for e in "$@"; do
    [ "$e" = "-" ] && E="" || E="$e"
    env $E timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('[$e] c2', d['value'], d['ms_per_step'])"
  done
done

#!/bin/bash
# c2 3-lane A/B over env settings on one build, interleaved: bash scripts/r05_ab_env.sh TAG "ENV1" "ENV2" ...
# (an ENV is 'A=1 B=2' or '-' for none); 300 det-batches each, two rounds
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05ab}
shift
mkdir -p $O
for rep in 1 2; do
  for e in "$@"; do
    [ "$e" = "-" ] && E="" || E="$e"
    env $E timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('[$e]', 'c2', d['value'], d['ms_per_step'])"
  done
done

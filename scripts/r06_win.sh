#!/bin/bash
# c2 short-window effects: 20 timed det-batches after 3 / 12 / 40 warm-up det-batches, and 100 after 3
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6win_${1:-a}
mkdir -p $O
for rep in 1 2; do
  for cfg in "20 3" "20 12" "20 40" "100 3"; do
    set -- $cfg
    timeout -k 10 300 python3 bench.py --steps $1 --warmup $2 --no-cpu-baseline --no-extras > $O/b.json 2> $O/b.err || exit $?
    python3 -c "import json; d=json.load(open('$O/b.json')); print('steps $1 warmup $2', d['value'], d['ms_per_step'], d['faces_per_frame'])"
  done
done

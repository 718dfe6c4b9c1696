#!/bin/bash
# lanes 4 / 5 / 6 (8 HW queues) on the default c2 run and on 20-det-batch windows, interleaved
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6ln_${1:-a}
mkdir -p $O
for rep in 1 2; do
  for L in 4 5 6; do
    timeout -k 10 400 python3 bench.py --lanes $L --no-cpu-baseline --no-extras --sustain-frames 10000 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('lanes $L c2 625', d['value'], d['ms_per_step'])"
  done
done
for rep in 1 2 3; do
  for L in 4 5 6; do
    timeout -k 10 300 python3 bench.py --lanes $L --steps 20 --warmup 3 --no-cpu-baseline --no-extras > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('lanes $L c2 20', d['value'], d['ms_per_step'])"
  done
done

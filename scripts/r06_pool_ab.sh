#!/bin/bash
# c2 driver-shaped line (20 steps) by frame source: cycled 32-frame pool vs distinct device frames
# with / without the page pre-touch; interleaved, then one default-length (10k frames) run
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6pool_${1:-a}
mkdir -p $O
for rep in 1 2; do
  for cfg in "32 1" "0 1" "0 0"; do
    set -- $cfg
    timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --pool $1 --touch $2 --no-cpu-baseline --no-extras > $O/b.json 2> $O/b.err || exit $?
    python3 -c "import json; d=json.load(open('$O/b.json')); print('pool $1 touch $2', d['value'], d['ms_per_step'], d['faces_per_frame'], d.get('sustained',{}).get('value'))"
  done
done
timeout -k 10 600 python3 bench.py --no-cpu-baseline --no-extras --sustain-frames 0 > $O/full.json 2> $O/full.err || exit $?
python3 -c "import json; d=json.load(open('$O/full.json')); print('default 10k frames pool 0', d['value'], d['ms_per_step'], d['faces_per_frame'])"

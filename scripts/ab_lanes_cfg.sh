#!/bin/bash
# lanes 3 / 4 for c3 and c5 (bench defaults otherwise: 8 HW queues), then the default c2 line
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/lc_${1:-a}
mkdir -p $O
for c in c3 c5; do
  for L in 3 4; do
    timeout -k 10 400 python3 bench.py --config $c --steps 60 --lanes $L --no-cpu-baseline --no-extras --sustain-frames 0 > $O/$c.json 2> $O/$c.err
    python3 -c "import json; d=json.load(open('$O/$c.json')); print('$c lanes=$L', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 400 python3 bench.py > $O/c2_default.json 2> $O/c2_default.err
python3 -c "import json; d=json.load(open('$O/c2_default.json')); print('c2 default', d['value'], d['ms_per_step'], d['config']['lanes'])"

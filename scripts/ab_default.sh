#!/bin/bash
# default bench (625 det-batches, no extras) vs the previous defaults (4 HW queues, 3 lanes), interleaved
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/abd_${1:-a}
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-extras > $O/new.json 2> $O/new.err
  python3 -c "import json; d=json.load(open('$O/new.json')); print('new (8 q, 4 lanes)', d['value'], d['ms_per_step'])"
  GPU_MAX_HW_QUEUES=4 timeout -k 10 400 python3 bench.py --lanes 3 --no-cpu-baseline --no-extras > $O/old.json 2> $O/old.err
  python3 -c "import json; d=json.load(open('$O/old.json')); print('old (4 q, 3 lanes)', d['value'], d['ms_per_step'])"
done

#!/bin/bash
# bench lines for BASELINE configs 3-5 (defaults: 10k frames for the detector configs)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/bc_${1:-a}
mkdir -p $O
for c in ${2:-c3 c4 c5}; do
    timeout -k 10 500 python3 bench.py --config $c > $O/$c.json 2> $O/$c.err
    python3 -c "import json; d=json.load(open('$O/$c.json')); print('$c', d['value'], d['ms_per_step'], d['roofline']['frac'], (d.get('cpu_baseline') or {}).get('value'))"
done

#!/bin/bash
# config 3 bench line (default length, CPU baseline) on the final tree
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c3_${1:-a}
mkdir -p $O
timeout -k 10 900 python3 bench.py --config c3 > $O/bench_c3.json 2> $O/bench_c3.err || { tail -5 $O/bench_c3.err; exit 1; }
python3 -c "
import json; d = json.load(open('$O/bench_c3.json'))
print('c3', d['value'], 'ms/step', d['ms_per_step'], 'faces/frame', d['faces_per_frame'], 'roof', d['roofline']['frac'], 'cpu', (d.get('cpu_baseline') or {}).get('value'), 'stagger', d['config']['lane_stagger_ms'])"

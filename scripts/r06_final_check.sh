#!/bin/bash
# driver-shaped check of the final tree: smoke, then `bench.py --gpus 1 --steps 20 --warmup 3`
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6fin_${1:-a}
mkdir -p $O
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -20 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 900 python3 bench.py --gpus 1 --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || { tail -20 $O/bench.err; exit 1; }
python3 -c "
import json; r = json.load(open('$O/bench.json'))
print('c2', r['value'], 'ms/step', r['ms_per_step'], 'faces/frame', r['faces_per_frame'], 'roof', r['roofline']['frac'], r['roofline']['avg_launch_ms'], 'sustained', r.get('sustained', {}).get('value'), 'cpu', r['cpu_baseline']['value'], r['config']['frame_source'][:40], r['config']['lane_stagger_ms'])"

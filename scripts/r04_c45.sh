#!/bin/bash
# config 5 (distinct device frames, grouping leg) and config 4 bench lines + a c4 kernel trace
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04c45}
mkdir -p $O
timeout -k 10 400 python3 bench.py --config c5 --no-cpu-baseline > $O/bench_c5.json 2> $O/bench_c5.err || exit $?
python3 -c "
import json; r = json.load(open('$O/bench_c5.json'))
print('c5', r['value'], 'ms/step', r['ms_per_step'], 'f/frame', r['faces_per_frame'], 'e2e', r['roofline_e2e']['frac'], 'grouping', {k: r['grouping'][k] for k in ('faces', 'clustered', 'clustered_frac', 'dedupe_s', 'sweep_s')})"
timeout -k 10 300 python3 bench.py --config c4 --no-cpu-baseline > $O/bench_c4.json 2> $O/bench_c4.err || exit $?
python3 -c "
import json; r = json.load(open('$O/bench_c4.json'))
print('c4', r['value'], 'ms/step', r['ms_per_step'], 'roof', r['roofline']['frac'], 'e2e', r['roofline_e2e']['frac'])"
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/raw -o run -- python3 bench.py --config c4 --steps 10 --warmup 3 --no-cpu-baseline > $O/c4_trace.json 2> $O/c4_trace.err || exit $?
python3 scripts/kstats.py $O/raw 20 > $O/c4_kernel_stats.txt 2>&1
rm -rf $O/raw
head -12 $O/c4_kernel_stats.txt

#!/bin/bash
# VR on both k_pnet launches: parity tests, per-launch rocprof rows VR off / on, phase clocks,
# then the driver-shaped c2 line on the make_frames-style device frames.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6vr2_${1:-a}
mkdir -p $O
VTF_PNET_VR=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py -k "mtcnn or pnet or nms" > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/tests.log | tail -2; grep -E "^FAILED|stage-1 cell" $O/tests.log | head
[ $rc -eq 0 ] || exit $rc
for vr in 0 1 0 1; do
  VTF_PNET_VR=$vr timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/t$vr -o run -- python3 -u scripts/probe_pnet.py child > $O/p$vr.txt 2> $O/p$vr.err || exit $?
  python3 - "$O/t$vr" "$vr" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)
rows = list(csv.DictReader(open(f[0]))) if f else []
print('vr', sys.argv[2], ' | '.join('%s %.1f us x%s' % (r['Name'].split('(')[0][-40:], float(r['AverageNs']) / 1e3, r['Calls']) for r in rows if 'k_pnet' in r['Name']))
PY
  rm -rf $O/t$vr
done
for vr in 0 1; do
  VTF_PNET_VR=$vr VTF_PNET_DEBUG=256 timeout -k 10 120 python3 -u scripts/probe_pnet.py child > $O/clk$vr.txt 2> $O/clk$vr.err || exit $?
  echo "clocks vr $vr: $(grep -i phase $O/clk$vr.err | tail -2 | tr '\n' ' ')"
done
timeout -k 10 900 python3 bench.py --steps 20 --warmup 3 > $O/bench.json 2> $O/bench.err || exit $?
python3 -c "
import json; r = json.load(open('$O/bench.json'))
print('bench', r['value'], 'ms/step', r['ms_per_step'], 'faces/frame', r.get('faces_per_frame'), 'roof', r['roofline']['frac'], r['roofline']['avg_launch_ms'], 'sustained', r.get('sustained', {}).get('value'), 'cpu', r['cpu_baseline']['value'], r['cpu_baseline']['repeats_s'])
print([ (s['stage'], s['bound_us']) for s in r['roofline_e2e']['stages']])"

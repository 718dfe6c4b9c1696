#!/bin/bash
# End-of-round evidence on one box: GPU tests + smoke, the default bench line (config 2), kernel
# traces (1 and 4 lanes), SQ / FETCH_SIZE / WRITE_SIZE passes (1 lane), dispatch counts, and the
# config 3 / 4 / 5 bench lines (with their CPU baselines).  bash scripts/profile_r06.sh TAG [skip-tests|main|configs]
# (skip-tests and main stop before the configs; tests: bash scripts/r06_check.sh)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/p6_${1:-a}
mkdir -p $O
if [ "${2:-}" != configs ]; then
if [ "${2:-}" != skip-tests ]; then
  timeout -k 10 800 python -u -m pytest -v -rA --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
  rc=$?
  grep -E "passed|failed|error" $O/tests.log | tail -2
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || exit $?
  tail -1 $O/smoke.log
fi
timeout -k 10 500 python3 bench.py > $O/bench_c2.json 2> $O/bench_c2.err || exit $?
python3 -c "
import json; r = json.load(open('$O/bench_c2.json'))
print('c2', r['value'], r['unit'], 'ms/step', r['ms_per_step'], 'faces/frame', r['faces_per_frame'], 'roof', r['roofline']['frac'], r['roofline']['avg_launch_ms'], 'sustained', r.get('sustained', {}).get('value'), 'cpu', r['cpu_baseline']['value'])"
B="--no-cpu-baseline --no-extras --sustain-frames 0"
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c2_trace -o run -- python3 bench.py --steps 10 --warmup 3 $B > $O/c2_trace.json 2> $O/c2_trace.err || exit $?
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c2_trace1 -o run -- python3 bench.py --steps 32 --warmup 3 --lanes 1 $B > $O/c2_trace1.json 2> $O/c2_trace1.err || exit $?
python3 scripts/kstats.py $O/c2_trace 40 > $O/c2_kernel_stats_4lane.txt 2>&1
python3 scripts/kstats.py $O/c2_trace1 70 > $O/c2_kernel_stats_1lane.txt 2>&1
python3 scripts/dispatch_counts.py $O/c2_trace1 > $O/dispatch_counts.txt 2>&1
timeout -s KILL 240 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $O/c2_pmc_sq -o run -- python3 bench.py --steps 3 --warmup 1 --lanes 1 $B > /dev/null 2> $O/c2_pmc_sq.err || exit $?
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/c2_pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --lanes 1 $B > /dev/null 2> $O/c2_pmc_fetch.err || exit $?
timeout -s KILL 240 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/c2_pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --lanes 1 $B > /dev/null 2> $O/c2_pmc_write.err || exit $?
python3 scripts/pmc_table.py $O c2 30 > $O/c2_pmc_table.txt 2>&1
find $O -name '*.csv' -size +5M -delete
find $O -name '*.db' -delete
head -8 $O/c2_kernel_stats_1lane.txt
python3 - $O <<'PY'
import json, re, sys
O = sys.argv[1]
r = json.load(open(O + '/bench_c2.json'))['roofline']
r1 = json.load(open(O + '/c2_trace1.json'))['roofline']
rows = [l for l in open(O + '/c2_kernel_stats_1lane.txt') if 'k_pnet' in l]
avg = sum(float(l.split()[-7]) for l in rows) / 1e3 if rows else 0
fl = r['flops_per_launch']
print('frac check: bench events %.4f ms -> %.4f; same-box 1-lane traced run events %.4f ms -> %.4f; its rocprof k_pnet rows %.4f ms -> %.4f'
      % (r['avg_launch_ms'], r['frac'], r1['avg_launch_ms'], r1['frac'], avg, fl / (avg / 1e3) / 1e12 / r['peak'] if avg else 0))
PY
cat $O/dispatch_counts.txt
head -6 $O/c2_pmc_table.txt
[ "${2:-}" = main ] || [ "${2:-}" = skip-tests ] && exit 0
fi
for c in c3 c4 c5; do
  timeout -k 10 600 python3 bench.py --config $c > $O/bench_$c.json 2> $O/bench_$c.err || exit $?
  python3 -c "
import json; d = json.load(open('$O/bench_$c.json'))
print('$c', d['value'], 'ms/step', d['ms_per_step'], 'roof', d['roofline']['frac'], 'cpu', (d.get('cpu_baseline') or {}).get('value'))"
done
echo profile-done

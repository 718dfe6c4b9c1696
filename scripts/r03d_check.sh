#!/bin/bash
# GPU tests, k_pnet A/B with counters (scripts/ab_pnet_pmc.sh), c2 3-lane A/B (base vs new build)
# and a one-lane kernel trace of the new build (blit / fill dispatch counts per det-batch).
# bash scripts/r03d_check.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ck_${1:-a}
mkdir -p $O
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?
tail -3 $O/tests.log
[ $rc -eq 0 ] || exit $rc
bash scripts/ab_pnet_pmc.sh ${1:-a} || exit $?
L=$PWD/video-to-faces_amd/lib
for rep in 1 2; do
  for lib in $L/libvtf_hip_base.so $L/libvtf_hip.so; do
    VTF_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$(basename $lib)', 'c2', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/trace -o run -- python3 bench.py --steps 32 --warmup 2 --lanes 1 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/trace_bench.json 2> $O/trace.err || exit $?
python3 scripts/kstats.py $O/trace 60 > $O/kstats_1lane.txt 2>&1 || true
rm -rf $O/trace
head -45 $O/kstats_1lane.txt

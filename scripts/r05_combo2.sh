#!/bin/bash
# round-5 combo 2: MTCNN / shape GPU tests (tiled resample), one-lane c2 trace + 3-lane occupancy,
# candidate front phase probe, c2 3-lane A/B (round-4 base vs this build)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05c2}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error|FAILED" $O/tests.log | tail -6
[ $rc -eq 0 ] || exit $rc
bash scripts/r04_c2trace.sh ${1:-r05c2}/tr > /dev/null || exit $?
grep -E "resample|sat_|cand_front|k_pnet" $O/tr/c2_kernel_stats_1lane.txt
B="--no-cpu-baseline --no-extras --sustain-frames 0"
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/tr3 -o run -- python3 bench.py --steps 48 --warmup 3 $B > $O/tr3.json 2> $O/tr3.err || exit $?
python3 scripts/busy.py $O/tr3 0.3 > $O/busy3.txt 2>&1; cat $O/busy3.txt
find $O/tr3 -name '*.db' -delete
bash scripts/probe_front.sh ${1:-r05c2} "0 1 2 4" 2>&1 | tail -8
BL=$PWD/video-to-faces_amd/lib/libvtf_hip_base.so
for rep in 1 2; do
  for v in base new; do
    [ $v = base ] && E="VTF_HIP_LIB=$BL" || E=""
    env $E timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$v', 'c2', d['value'], d['ms_per_step'])"
  done
done

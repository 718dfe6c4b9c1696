#!/bin/bash
# MTCNN / box GPU tests on the new build, k_pnet solo and c2 3-lane A/B of base / new /
# new + VTF_PNET_CONC=1, and the steady-state dispatch counts of a one-lane trace.
# bash scripts/r03e_check.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ce_${1:-a}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py tests/test_boxes.py tests/test_yolo_gpu.py > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
L=$PWD/video-to-faces_amd/lib
for rep in 1 2 3; do
  for v in base new conc; do
    lib=$L/libvtf_hip.so; [ $v = base ] && lib=$L/libvtf_hip_base.so
    c=0; [ $v = conc ] && c=1
    VTF_PNET_CONC=$c VTF_HIP_LIB=$lib timeout -k 10 120 python3 -u scripts/probe_pnet.py child > $O/t.txt 2> $O/t.err || exit $?
    echo "$v pnet $(tail -1 $O/t.txt)"
  done
done
for rep in 1 2; do
  for v in base new conc; do
    lib=$L/libvtf_hip.so; [ $v = base ] && lib=$L/libvtf_hip_base.so
    c=0; [ $v = conc ] && c=1
    VTF_PNET_CONC=$c VTF_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$v', 'c2', d['value'], d['ms_per_step'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/trace -o run -- python3 bench.py --steps 32 --warmup 2 --lanes 1 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/trace_bench.json 2> $O/trace.err || exit $?
python3 scripts/dispatch_counts.py $O/trace > $O/dispatch_counts.txt 2>&1
python3 scripts/kstats.py $O/trace 60 > $O/kstats_1lane.txt 2>&1
rm -rf $O/trace
cat $O/dispatch_counts.txt

#!/bin/bash
# MTCNN GPU tests, k_pnet solo A/B of VTF_PNET_PR=0 (base) vs 1 (new), 3 rounds, phase
# clocks per variant of the new build, c2 3-lane A/B (2 rounds).  bash scripts/r03g_check.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ch_${1:-a}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py > $O/tests.log 2>&1
rc=$?
tail -2 $O/tests.log
[ $rc -eq 0 ] || exit $rc
L=$PWD/video-to-faces_amd/lib
for rep in 1 2 3; do
  for v in base new; do
    lib=$L/libvtf_hip.so; pr=1; [ $v = base ] && pr=0
    VTF_PNET_PR=$pr VTF_HIP_LIB=$lib timeout -k 10 120 python3 -u scripts/probe_pnet.py child > $O/t.txt 2> $O/t.err || exit $?
    echo "$v pnet $(tail -1 $O/t.txt)"
  done
done
VTF_PNET_DEBUG=256 timeout -k 10 120 python3 -u scripts/probe_pnet.py child > $O/clk.txt 2> $O/clk.err || exit $?
grep -A2 "phase clocks" $O/clk.err | tail -3
for rep in 1 2; do
  for v in base new; do
    lib=$L/libvtf_hip.so; pr=1; [ $v = base ] && pr=0
    VTF_PNET_PR=$pr VTF_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$v', 'c2', d['value'], d['ms_per_step'])"
  done
done

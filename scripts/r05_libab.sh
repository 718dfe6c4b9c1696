#!/bin/bash
# MTCNN GPU tests on the working build, then k_pnet solo timing and c2 A/B against
# lib/libvtf_hip_base.so, interleaved on one box: bash scripts/r05_libab.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05lab}
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
BASE="VTF_HIP_LIB=$GRAFT_REPO_ROOT/video-to-faces_amd/lib/libvtf_hip_base.so"
for rep in 1 2; do
  for v in base new; do
    [ $v = base ] && E="$BASE" || E=""
    env $E timeout -k 10 200 python3 scripts/probe_pnet.py child > $O/probe.txt 2> $O/probe.err || exit $?
    echo "$v pnet $(tail -1 $O/probe.txt)"
  done
done
for rep in 1 2; do
  for v in base new; do
    [ $v = base ] && E="$BASE" || E=""
    env $E timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$v', 'c2', d['value'], d['ms_per_step'])"
  done
done

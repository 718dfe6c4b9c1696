#!/bin/bash
# NMS v2 check: NMS-using GPU tests on the new build, NMS timing base vs new, one-lane c2 trace of
# the new build, c2 3-lane A/B (base = lib/libvtf_hip_base.so)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05nms}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v -rA --timeout 300 --timeout-method thread -m gpu tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py tests/test_rcnn_gpu.py tests/test_yolo_gpu.py > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/tests.log | tail -3
[ $rc -eq 0 ] || exit $rc
B=$PWD/video-to-faces_amd/lib/libvtf_hip_base.so
N=$PWD/video-to-faces_amd/lib/libvtf_hip.so
for lib in $B $N; do
  VTF_HIP_LIB=$lib timeout -k 10 200 python3 scripts/nms_time.py 20 > $O/time_$(basename $lib .so).log 2>&1 || exit $?
  echo "$(basename $lib)"; grep "^n " $O/time_$(basename $lib .so).log
done
bash scripts/r04_c2trace.sh ${1:-r05nms}/tr || exit $?
for rep in 1 2; do
  for lib in $B $N; do
    VTF_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$(basename $lib)', 'c2', d['value'], d['ms_per_step'])"
  done
done

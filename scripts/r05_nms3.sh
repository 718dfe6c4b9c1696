#!/bin/bash
# NMS tie-order fix without host copies: NMS-using GPU tests, one-lane c2 trace (dispatch counts), c2 A/B
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05nms3}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py tests/test_rcnn_gpu.py tests/test_yolo_gpu.py tests/test_facenet_gpu.py > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error|FAILED" $O/tests.log | tail -8
[ $rc -eq 0 ] || exit $rc
bash scripts/r04_c2trace.sh ${1:-r05nms3}/tr || exit $?
cat $O/tr/dispatch_counts.txt
B=$PWD/video-to-faces_amd/lib/libvtf_hip_base.so
N=$PWD/video-to-faces_amd/lib/libvtf_hip.so
for rep in 1 2; do
  for lib in $B $N; do
    VTF_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$(basename $lib)', 'c2', d['value'], d['ms_per_step'])"
  done
done

#!/bin/bash
# round-5 combo: GPU tests (MTCNN/shapes/RCNN/YOLO/FaceNet), FaceNet Block17 split timing, one-lane
# c2 trace + dispatch counts, c2 3-lane A/B: base lib, new lib, new lib + VTF_PNET_PRIO=1
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05c1}
mkdir -p $O
timeout -k 10 700 python -u -m pytest -q -s --timeout 300 --timeout-method thread -m gpu tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py tests/test_rcnn_gpu.py tests/test_yolo_gpu.py tests/test_facenet_gpu.py > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error|FAILED|fused vs" $O/tests.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python3 scripts/facenet_time.py 20 "VTF_B17_SPLIT=1,VTF_B17_SPLIT=0" > $O/fn_time.txt 2>&1 || exit $?
cat $O/fn_time.txt
bash scripts/r04_c2trace.sh ${1:-r05c1}/tr > /dev/null || exit $?
cat $O/tr/dispatch_counts.txt; head -8 $O/tr/c2_kernel_stats_1lane.txt
B=$PWD/video-to-faces_amd/lib/libvtf_hip_base.so
for rep in 1 2; do
  for v in base new prio; do
    case $v in base) E="VTF_HIP_LIB=$B";; new) E="";; prio) E="VTF_PNET_PRIO=1";; esac
    env $E timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$v', 'c2', d['value'], d['ms_per_step'])"
  done
done

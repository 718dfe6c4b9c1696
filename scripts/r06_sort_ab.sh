#!/bin/bash
# small-footprint tile sort + raw conv1 pooling max: parity tests, then same-box A/B vs the
# committed library (k_pnet solo, c2 20 / 300 det-batches), then a 4-lane trace of the new one
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6sort_${1:-a}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py tests/test_rcnn_gpu.py -k "mtcnn or nms or pnet or rcnn or rpn or roi or iom or config" > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/tests.log | tail -2; grep -E "^FAILED|stage-1 cell" $O/tests.log | head
[ $rc -eq 0 ] || exit $rc
B=$PWD/video-to-faces_amd/lib/libvtf_hip_base.so
N=$PWD/video-to-faces_amd/lib/libvtf_hip.so
for rep in 1 2; do
  for lib in $B $N; do
    VTF_HIP_LIB=$lib timeout -k 10 120 python3 -u scripts/probe_pnet.py child > $O/p.txt 2> $O/p.err || exit $?
    echo "$(basename $lib) pnet $(tail -1 $O/p.txt)"
  done
done
for rep in 1 2 3; do
  for lib in $B $N; do
    VTF_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$(basename $lib) c2 20', d['value'], d['ms_per_step'], d['faces_per_frame'])"
  done
done
for rep in 1 2; do
  for lib in $B $N; do
    VTF_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 300 --warmup 3 --no-cpu-baseline --no-extras > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$(basename $lib) c2 300', d['value'], d['ms_per_step'], d['faces_per_frame'])"
  done
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t4 -o run -- python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > $O/t4.json 2> $O/t4.err || exit $?
python3 scripts/kstats.py $O/t4 60 | grep -v "at::native" | head -24 > $O/k4.txt; cat $O/k4.txt
find $O -name '*.db' -delete
bash scripts/r06_win.sh ${1:-a} || exit $?

#!/bin/bash
# A/B of two builds on one box (lib/libvtf_hip_base.so vs lib/libvtf_hip.so): GPU tests on the new
# build, 1-lane kernel stats of both, c2 3-lane bench interleaved:  bash scripts/ab_lib_k.sh TAG PATTERN
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-a}; PAT=${2:-span}
O=gpurun_out/abk_$TAG
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py > $O/tests.log 2>&1
tail -1 $O/tests.log
B=$PWD/video-to-faces_amd/lib/libvtf_hip_base.so
N=$PWD/video-to-faces_amd/lib/libvtf_hip.so
for lib in $B $N; do
  t=$(basename $lib .so)
  VTF_HIP_LIB=$lib bash scripts/kprof.sh ${TAG}_$t c2 --lanes 1
  grep -E "$PAT" gpurun_out/kp_${TAG}_$t/kernel_stats.txt | sed "s/^/$t /" | cut -c1-150
done
for rep in 1 2; do
  for lib in $B $N; do
    VTF_HIP_LIB=$lib timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-extras > $O/c2.json 2> $O/c2.err
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$(basename $lib)', 'c2', d['value'], d['ms_per_step'])"
  done
done

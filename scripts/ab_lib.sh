#!/bin/bash
# A/B of two builds on one box: lib/libvtf_hip_base.so (before) vs lib/libvtf_hip.so (after):
# GPU tests on the new build, k_pnet solo (probe_pnet child) and c2 3-lane bench, interleaved
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ab_${1:-a}
TESTS=${2:-"tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py"}
mkdir -p $O
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread $TESTS > $O/tests.log 2>&1
tail -1 $O/tests.log
B=$PWD/video-to-faces_amd/lib/libvtf_hip_base.so
N=$PWD/video-to-faces_amd/lib/libvtf_hip.so
for rep in 1 2; do
  for lib in $B $N; do
    VTF_HIP_LIB=$lib timeout -k 10 120 python3 -u scripts/probe_pnet.py child > $O/pnet.txt 2> $O/pnet.err
    echo "$(basename $lib) pnet $(tail -1 $O/pnet.txt)"
  done
done
for rep in 1 2; do
  for lib in $B $N; do
    VTF_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$(basename $lib)', 'c2', d['value'], d['ms_per_step'])"
  done
done

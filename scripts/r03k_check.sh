#!/bin/bash
# MTCNN GPU tests on the 12-byte SAT build, then one-lane kernel traces of base / new (SAT passes, resample, candidate crops).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ck_${1:-a}
mkdir -p $O
VTF_HIP_LIB=$PWD/video-to-faces_amd/lib/libvtf_hip_sat3.so timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py > $O/tests.log 2>&1
rc=$?
tail -1 $O/tests.log
[ $rc -eq 0 ] || exit $rc
for v in base new; do
  lib=$PWD/video-to-faces_amd/lib/libvtf_hip_sat3.so; [ $v = base ] && lib=$PWD/video-to-faces_amd/lib/libvtf_hip_base.so
  VTF_HIP_LIB=$lib timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/$v -o run -- python3 bench.py --steps 16 --warmup 2 --lanes 1 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/$v.json 2> $O/$v.err || exit $?
  python3 scripts/kstats.py $O/$v 60 > $O/kstats_$v.txt; rm -rf $O/$v
  grep -E "k_pnet|resample|sat_|cand" $O/kstats_$v.txt | sed "s/^/$v /"
  python3 -c "import json; d=json.load(open('$O/$v.json')); print('$v 1-lane under tracer', d['value'], d['ms_per_step'])"
done

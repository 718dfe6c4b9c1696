#!/bin/bash
# RNet span-pool FNU A/B: MTCNN GPU tests on the working build, the k_cand_front_w24 kernel time
# of both builds (one-lane kernel trace), then c2 interleaved against lib/libvtf_hip_base.so.
# bash scripts/r05_front_ab.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05span}
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py > $O/tests.log 2>&1
rc=$?; tail -2 $O/tests.log; [ $rc -eq 0 ] || exit $rc
B="--no-cpu-baseline --no-extras --sustain-frames 0"
for v in base new; do
  if [ $v = base ]; then export VTF_HIP_LIB=$GRAFT_REPO_ROOT/video-to-faces_amd/lib/libvtf_hip_base.so; else unset VTF_HIP_LIB; fi
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/tr_$v -o run -- python3 bench.py --steps 32 --warmup 3 --lanes 1 $B > $O/tr_$v.json 2> $O/tr_$v.err || exit $?
  python3 scripts/kstats.py $O/tr_$v 60 > $O/kstats_$v.txt 2>&1
  echo "== $v"; echo "$(grep -E 'k_conv_span_pool' $O/kstats_$v.txt)"
done
unset VTF_HIP_LIB
find $O -name '*.db' -delete
for rep in 1 2; do
  for v in base new; do
    if [ $v = base ]; then export VTF_HIP_LIB=$GRAFT_REPO_ROOT/video-to-faces_amd/lib/libvtf_hip_base.so; else unset VTF_HIP_LIB; fi
    timeout -k 10 300 python3 bench.py --steps 300 $B > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$v', 'c2', d['value'], d['ms_per_step'])"
  done
done

#!/bin/bash
# bin averages by fma-corrected reciprocals: MTCNN / shape GPU tests, then same-box A/B vs HEAD
# (RNet / ONet front kernel times from a 1-lane trace each, c2 20 / 625 det-batches)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6ba_${1:-a}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py -k "mtcnn or sat or detect or resample or front or rnet or onet or cand" > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/tests.log | tail -2; grep -E "^FAILED" $O/tests.log | head
[ $rc -eq 0 ] || exit $rc
B=$PWD/video-to-faces_amd/lib/libvtf_hip_base.so
N=$PWD/video-to-faces_amd/lib/libvtf_hip.so
for lib in $B $N; do
  VTF_HIP_LIB=$lib timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t -o run -- python3 bench.py --steps 32 --warmup 3 --lanes 1 --no-cpu-baseline --no-extras > $O/t.json 2> $O/t.err || exit $?
  echo "== $(basename $lib)"; python3 scripts/kstats.py $O/t 80 | grep -E "k_cand_front|k_resample|k_pnet" | cut -c1-100
  rm -rf $O/t
done
for rep in 1 2 3 4; do
  for lib in $B $N; do
    VTF_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$(basename $lib) c2 20', d['value'], d['ms_per_step'])"
  done
done
for rep in 1 2; do
  for lib in $B $N; do
    VTF_HIP_LIB=$lib timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-extras --sustain-frames 10000 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$(basename $lib) c2 625', d['value'], d['ms_per_step'])"
  done
done

#!/bin/bash
# ONet front-end band height A/B (VTF_FRONT_PB = 1 / 2 / 3): MTCNN tests at each, c2 3-lane bench
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fpb_${1:-a}
mkdir -p $O
for pb in 2 3; do
  VTF_FRONT_PB=$pb timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mtcnn_gpu.py -k "720p or small or span" > $O/tests_$pb.log 2>&1
  echo "pb=$pb $(tail -1 $O/tests_$pb.log)"
done
for rep in 1 2; do
  for pb in 1 2 3; do
    VTF_FRONT_PB=$pb timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('pb=$pb', 'c2', d['value'], d['ms_per_step'])"
  done
done
for pb in 1 2 3; do
  VTF_FRONT_PB=$pb bash scripts/kprof.sh fpb$pb c2 --lanes 1
  echo "pb=$pb $(grep 'k_cand_frontILi48' gpurun_out/kp_fpb$pb/kernel_stats.txt)"
done

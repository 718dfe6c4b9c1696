#!/bin/bash
# split conv tile A/B on c2: 128x64 @3/CU vs 256x64 @2/CU vs k_conv staging-split
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ms2_${1:-a}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mtcnn_gpu.py > $O/tests.log 2>&1
tail -1 $O/tests.log
for rep in 1 2; do
for arm in "1 128" "1 256" "0 128"; do
  set -- $arm
  VTF_MTCNN_SP=$1 VTF_DMA_SPLIT64=$2 timeout -k 10 300 python3 bench.py --steps 200 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err
  python3 -c "import json; d=json.load(open('$O/c2.json')); print('c2 sp=$1 tile=$2', d['value'], d['ms_per_step'])"
done
done
bash scripts/kprof.sh ms2_${1:-a}_k c2 --lanes 1
grep -E "dma|cand_front|maxpool_ks" gpurun_out/kp_ms2_${1:-a}_k/kernel_stats.txt

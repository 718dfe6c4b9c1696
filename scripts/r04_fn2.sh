#!/bin/bash
# FaceNet fused blocks: timing + Block17 stage clocks
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04fn2}
mkdir -p $O
timeout -k 10 200 python3 scripts/facenet_time.py 20 > $O/time.log 2>&1 || exit $?
cat $O/time.log
VTF_B17_CLK=1 timeout -k 10 200 python3 scripts/facenet_time.py 1 1 > $O/clk.log 2>&1 || exit $?
grep "k_block17 cycles" $O/clk.log | tail -3

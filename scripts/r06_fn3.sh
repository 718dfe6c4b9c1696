#!/bin/bash
# FaceNet: Block17 per-image stage 4 (VTF_B17_SPLIT=0) vs the batch tail launch, both on padded weights
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6fn3_${1:-a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_facenet_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 300 python3 -u scripts/r06_b17ws.py 20 "VTF_B17_SPLIT=1,VTF_B17_SPLIT=0,VTF_FN_WPAD=0+VTF_B17_SPLIT=0,VTF_FN_WPAD=0+VTF_B17_SPLIT=1" facenet > $O/ab.txt 2> $O/ab.err || exit $?
cat $O/ab.txt

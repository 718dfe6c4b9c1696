#!/bin/bash
# FaceNet padded weight strides (build-time VTF_FN_WPAD): GPU tests, A/B (bitwise), layer listing
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6fn2_${1:-a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_facenet_gpu.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 300 python3 -u scripts/r06_b17ws.py 20 "VTF_FN_WPAD=0,VTF_FN_WPAD=112,VTF_FN_WPAD=8,VTF_FN_WPAD=56" facenet > $O/ab.txt 2> $O/ab.err || exit $?
cat $O/ab.txt
bash scripts/facenet_layers.sh r6fn2_${1:-a}_layers > /dev/null 2>&1 || exit $?
head -40 gpurun_out/fn_r6fn2_${1:-a}_layers/layers.txt

#!/bin/bash
# k_pnet merged-chain conv1 (16x16x32, main + cross in one chain) vs the 32x32 [w0 | w1] layout
# (VTF_PNET_C1K=0): MTCNN GPU tests, k_pnet solo timing, c2 A/B (interleaved, one box)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05c1k}
mkdir -p $O
timeout -k 10 500 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for e in 1 0; do
    VTF_PNET_C1K=$e timeout -k 10 200 python3 scripts/probe_pnet.py child > $O/probe.txt 2> $O/probe.err || exit $?
    echo "C1K=$e $(tail -1 $O/probe.txt)"
  done
done
bash scripts/r05_ab_env.sh ${1:-r05c1k}_ab "-" "VTF_PNET_C1K=0"

#!/bin/bash
# round-5 parity items: classify in sklearn's bits, fused FaceNet bit identity, device crops without
# exemptions, the split-fp16 GEMM bounds
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05par}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -v -rA -s --timeout 300 --timeout-method thread -m gpu tests/test_grouping_gpu.py tests/test_facenet_gpu.py tests/test_gemm_split_gpu.py "tests/test_shapes_gpu.py::test_mtcnn_b16_device_crops" > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error|FAILED" $O/tests.log | tail -8
exit $rc

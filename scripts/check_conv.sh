#!/bin/bash
# conv change check: encoder/detector GPU tests + 1/3-lane benches + 1-lane kernel stats
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/conv_${1:-a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_facenet_gpu.py tests/test_yolo_gpu.py tests/test_rcnn_gpu.py tests/test_vit_gpu.py tests/test_mtcnn_gpu.py > $O/tests.log 2>&1
timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --lanes 1 --no-cpu-baseline > $O/bench_l1.json 2> $O/bench_l1.err
timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench_l3.json 2> $O/bench_l3.err
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 --lanes 1 --no-cpu-baseline > $O/prof_bench.json 2> $O/prof.err
echo done

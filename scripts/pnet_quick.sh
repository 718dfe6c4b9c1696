#!/bin/bash
# k_pnet change check: MTCNN GPU parity tests, phase timings, default bench line
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pq_${1:-a}
MASKS=${2:-"0 1 2 8"}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 120 --timeout-method thread -m gpu tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py -k "mtcnn or pnet" > $O/tests.log 2>&1
timeout -k 10 300 python3 -u scripts/probe_pnet.py $MASKS > $O/masks.txt 2> $O/masks.err
VTF_PNET_DEBUG=256 timeout -k 10 120 python3 -u scripts/probe_pnet.py child > $O/clk_run.txt 2> $O/clk.txt
timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/bench.json 2> $O/bench.err
tail -3 $O/tests.log; cat $O/masks.txt; grep phase $O/clk.txt | tail -2; cut -c1-300 $O/bench.json

#!/bin/bash
# Kernel-trace + PMC profiles of the bench workloads (run on the GPU box via gpurun).
# Outputs under gpurun_out/prof_<tag>/; summarise with scripts/kstats.py / scripts/pmc_summary.py.
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
TAG=${1:-r01}
O=gpurun_out/prof_$TAG
mkdir -p $O
# the default bench command (MTCNN + FaceNet, 3 lanes) under the kernel tracer
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/mtcnn -o run -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > $O/mtcnn_bench.json 2> $O/mtcnn.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/yolo -o run -- python3 bench.py --det-model yolo --steps 5 --warmup 2 --no-cpu-baseline > $O/yolo_bench.json 2> $O/yolo.err
# HBM bytes of k_pnet: separate FETCH_SIZE / WRITE_SIZE passes (one lane: no co-running kernels)
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d $O/pmc_fetch -o run -- python3 bench.py --steps 3 --warmup 1 --lanes 1 --no-cpu-baseline > /dev/null 2> $O/pmc_fetch.err
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d $O/pmc_write -o run -- python3 bench.py --steps 3 --warmup 1 --lanes 1 --no-cpu-baseline > /dev/null 2> $O/pmc_write.err
echo profile-done

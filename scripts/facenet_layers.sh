#!/bin/bash
# FaceNet encoder-only (batch 128) under the kernel tracer: per-launch listing of one forward
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fn_$1
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 bench.py --config c4 --enc-model facenet --enc-precision ${2:-bf16} --steps 6 --warmup 2 --no-cpu-baseline > $O/bench.json 2> $O/err.txt
rc=$?
python3 scripts/fwd_layers.py $O/raw full > $O/layers.txt 2>&1
rm -rf $O/raw
exit $rc

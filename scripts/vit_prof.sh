#!/bin/bash
# ViT-L c4 under the kernel tracer: per-kind / per-grid durations of one forward
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/vp_$1
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 bench.py --config c4 --steps 6 --warmup 2 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/bench.json 2> $O/err.txt
rc=$?
python3 scripts/vit_layers.py $O/raw > $O/layers.txt 2>&1
rm -rf $O/raw
cat $O/layers.txt
exit $rc

#!/bin/bash
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cp_$1
mkdir -p $O
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/raw -o run -- python3 scripts/mtcnn_stats.py 3 > $O/run.txt 2>&1
python3 scripts/cand_layers.py $O/raw > $O/layers.txt 2>&1
rm -rf $O/raw
cat $O/layers.txt

#!/bin/bash
# YOLO per-launch listing of one c3 det-batch (1 lane)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6yl_${1:-a}
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace -d $O/t -o run -- python3 bench.py --config c3 --steps 6 --warmup 2 --lanes 1 --no-cpu-baseline --no-extras > $O/b.json 2> $O/b.err || exit $?
python3 scripts/yolo_layers.py $O/t > $O/layers.txt 2>&1
rm -rf $O/t
cat $O/layers.txt | tail -90

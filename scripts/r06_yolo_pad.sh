#!/bin/bash
# YOLO bf16x3 conv operand strides: B (weight rows) pad A/B by events; A (pixel) pad by kernel stats
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6yp_${1:-a}
mkdir -p $O
timeout -k 10 300 python3 -u scripts/r06_yolo_ab.py 5 "VTF_DMA3_BPAD=0,VTF_DMA3_BPAD=16,VTF_DMA3_BPAD=48,VTF_DMA3_BPAD=96" > $O/b.txt 2> $O/b.err || { tail -5 $O/b.err; exit 1; }
cat $O/b.txt
for ap in 0 16 48; do
  VTF_DMA3_APAD=$ap timeout -k 10 200 rocprofv3 --kernel-trace -d $O/pa$ap -o run -- python3 -u scripts/r06_yolo_ab.py 3 "VTF_DMA3_BPAD=0" > $O/pa$ap.txt 2> $O/pa$ap.err || exit $?
  echo "== A pad $ap"; python3 scripts/kstats.py $O/pa$ap 8 | cut -c1-100
done
find $O -name '*.db' -delete

#!/bin/bash
# one-lane config-2 kernel trace (32 det-batches) -> kernel stats; prints the top rows and the NMS rows
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r04tr}
mkdir -p $O
B="--no-cpu-baseline --no-extras --sustain-frames 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/c2_trace1 -o run -- python3 bench.py --steps 32 --warmup 3 --lanes 1 $B > $O/c2_trace1.json 2> $O/c2_trace1.err || exit $?
python3 scripts/kstats.py $O/c2_trace1 70 > $O/c2_kernel_stats_1lane.txt 2>&1
python3 scripts/dispatch_counts.py $O/c2_trace1 > $O/dispatch_counts.txt 2>&1
find $O -name '*.db' -delete
rm -rf $O/c2_trace1
head -12 $O/c2_kernel_stats_1lane.txt
grep -E "nms|iou|rocprim|seg_|plan|scatter|compact|flag|call_kept|tie" $O/c2_kernel_stats_1lane.txt
tail -1 $O/c2_kernel_stats_1lane.txt

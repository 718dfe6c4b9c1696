#!/bin/bash
# k_cand_front phase-skip probe: kernel time per VTF_FRONT_DEBUG mask (1 crop, 2 conv1, 4 pool)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pf_${1:-a}
mkdir -p $O
for m in ${2:-0 1 2 4 6 7}; do
    VTF_FRONT_DEBUG=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/raw_$m -o run -- python3 scripts/mtcnn_stats.py 3 > $O/run_$m.txt 2>&1
    python3 scripts/kstats.py $O/raw_$m 40 > $O/stats_$m.txt 2>&1
    rm -rf $O/raw_$m
    echo "mask $m"; grep cand_front $O/stats_$m.txt
done

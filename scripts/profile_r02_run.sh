#!/bin/bash
# profile_r02.sh + on-box summaries (the raw traces exceed gpurun's 64 MiB copy-back).
set -o pipefail
TAG=${1:-r02}
shift || true
CFGS=${@:-c2 c3 c4}
bash scripts/profile_r02.sh $TAG $CFGS > gpurun_out/prof_$TAG.log 2>&1
rc=$?
O=gpurun_out/prof_$TAG
for c in $CFGS; do
  python3 scripts/kstats.py $O/${c}_trace 30 > $O/${c}_kernel_stats.txt 2>&1
  python3 scripts/kstats.py $O/${c}_trace1 30 > $O/${c}_kernel_stats_1lane.txt 2>&1
  python3 scripts/pmc_table.py $O $c 20 > $O/${c}_pmc_table.txt 2>&1
  cp $O/${c}_trace.json $O/${c}_trace1.json $O/ 2>/dev/null
done
for c in $CFGS; do rm -rf $O/${c}_trace $O/${c}_trace1 $O/${c}_pmc_sq $O/${c}_pmc_fetch $O/${c}_pmc_write; done
du -sh gpurun_out
exit $rc

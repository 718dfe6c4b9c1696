#!/bin/bash
# k_pnet phase-skip times (VTF_PNET_DEBUG masks, candidate output off via bit 16) on one box,
# the X and PR launches separately via rocprofv3 kernel stats of the probe child.
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6pm_${1:-a}
MASKS=${2:-"16 17 18 20 24 48 80 127"}
mkdir -p $O
for m in $MASKS; do
  VTF_PNET_DEBUG=$m timeout -k 10 120 rocprofv3 --kernel-trace --stats -d $O/m$m -o run -- python3 -u scripts/probe_pnet.py child > $O/m$m.txt 2> $O/m$m.err || exit $?
  python3 - "$O/m$m" "$m" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)
rows = list(csv.DictReader(open(f[0]))) if f else []
ks = {r['Name']: r for r in rows if 'k_pnet' in r['Name']}
print('mask', sys.argv[2], ' '.join('%s %.1f us x%s' % (n.split('<')[1].split('>')[0].replace(' ', ''), float(r['AverageNs']) / 1e3, r['Calls']) for n, r in sorted(ks.items())))
PY
  tail -1 $O/m$m.txt
done
find $O -name '*.db' -delete

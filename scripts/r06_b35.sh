#!/bin/bash
# Block35 branches: input row-stride padding (per-call copy, experiment) -> k_block35_br kernel time
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6b35_${1:-a}
mkdir -p $O
timeout -k 10 200 python3 -u scripts/r06_b17ws.py 3 "VTF_B35_XPAD=0,VTF_B35_XPAD=8,VTF_B35_XPAD=56" facenet > $O/ab.txt 2> $O/ab.err || exit $?
cat $O/ab.txt
for xp in 0 8 56; do
  VTF_B35_XPAD=$xp timeout -k 10 200 rocprofv3 --kernel-trace -d $O/x$xp -o run -- python3 -u scripts/r06_b17ws.py 5 "VTF_B35_XPAD=$xp" facenet > $O/x$xp.txt 2> $O/x$xp.err || exit $?
  echo "== X pad $xp"; python3 scripts/kstats.py $O/x$xp 40 | grep -E "block35|block17|block8|kernel" | cut -c1-100
done
find $O -name '*.db' -delete

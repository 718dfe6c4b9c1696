#!/bin/bash
# NOTE: VTF_PNET_DEBUG 512 / 1024 existed only in the probe build of this experiment (profiles/r06_pnet_ldsconf_phases.txt)
# k_pnet conv2 LDS-conflict probes (VTF_PNET_DEBUG 512: 4-byte operand reads at one tap; 1024: the
# 16-byte ones; results wrong, timing and counters only): pair solo by events + conflict counters
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6c2p_${1:-a}
mkdir -p $O
for rep in 1 2; do
  for m in 16 528 1040 1552; do
    VTF_PNET_DEBUG=$m timeout -k 10 120 python3 -u scripts/probe_pnet.py child > $O/p.txt 2> $O/p.err || exit $?
    echo "rep $rep $(tail -1 $O/p.txt)"
  done
done
bash scripts/r06_pnet_ldsconf.sh c2p_${1:-a} "16 528 1040 1552" || exit $?

#!/bin/bash
# k_pnet sensitivity probes: solo time per VTF_PNET_DEBUG mask (timing-only extra work per
# resource: 512 conv1 MFMA, 1024 conv1 LDS reads, 2048 conv3 MFMA, 4096 conv3 LDS reads,
# 8192 conv3 epilogue VALU) plus phase-skip masks.  bash scripts/pnet_sens.sh TAG "masks"
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ps_${1:-a}
mkdir -p $O
timeout -k 10 500 python3 -u scripts/probe_pnet.py ${2:-0 512 1024 2048 4096 8192 0} > $O/masks.txt 2> $O/masks.err
cat $O/masks.txt

#!/bin/bash
# phase-skip probe of the fused candidate kernel on a fixed det-batch (stage counts printed)
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for m in ${MASKS:-0 1 2 4 8 16 31}; do
  VTF_CAND_DEBUG=$m timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/pc_raw -o run -- python3 scripts/probe_cand.py 5 > gpurun_out/pc_out.txt 2>&1
  echo "mask $m $(grep stats gpurun_out/pc_out.txt)"; python3 scripts/kstats.py gpurun_out/pc_raw 40 | grep -E "cand_fused|cand_front|k_conv<float"
  rm -rf gpurun_out/pc_raw
done

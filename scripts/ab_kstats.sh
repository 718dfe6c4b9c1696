#!/bin/bash
# per-kernel solo times of k_pnet (probe_pnet child under rocprofv3 --kernel-trace --stats) for
# lib/libvtf_hip_base.so vs lib/libvtf_hip.so.  bash scripts/ab_kstats.sh TAG
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/ak_${1:-a}
mkdir -p $O
for lib in base new; do
  L=$PWD/video-to-faces_amd/lib/libvtf_hip.so
  [ $lib = base ] && L=$PWD/video-to-faces_amd/lib/libvtf_hip_base.so
  VTF_HIP_LIB=$L timeout -k 10 180 rocprofv3 --kernel-trace --stats -d $O/$lib -o run --output-format csv -- python3 scripts/probe_pnet.py child > $O/$lib.txt 2> $O/$lib.err
  f=$(find $O/$lib -name '*kernel_stats.csv' | head -1)
  echo "== $lib"; grep k_pnet $f | cut -d, -f1-5
done

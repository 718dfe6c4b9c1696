#!/bin/bash
# A/B of library variants on the default bench, interleaved: bash scripts/ab_libs.sh <rounds> <lib names...>
set -e
cd "$GRAFT_REPO_ROOT"
R=$1; shift
mkdir -p gpurun_out/ab
for r in $(seq 1 $R); do
  for v in "$@"; do
    VTF_HIP_LIB=$PWD/video-to-faces_amd/lib/$v timeout -k 10 200 python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/ab/${v}_$r.json 2>/dev/null
  done
done
echo ab-done

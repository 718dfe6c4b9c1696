#!/bin/bash
# One-lane c2 A/B of the round's start (lib/libvtf_hip_old.so, 069f5d2) vs the current build (host
# round trips), then k_pnet phase clocks per variant of the current build.
# bash scripts/r03f_check.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cf_${1:-a}
mkdir -p $O
L=$PWD/video-to-faces_amd/lib
for rep in 1 2; do
  for v in old new; do
    lib=$L/libvtf_hip.so; [ $v = old ] && lib=$L/libvtf_hip_old.so
    VTF_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 200 --lanes 1 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$v', '1-lane c2', d['value'], 'faces/s', d['ms_per_step'], 'ms/step')"
  done
done
VTF_PNET_DEBUG=256 timeout -k 10 120 python3 -u scripts/probe_pnet.py child > $O/clk.txt 2> $O/clk.err || exit $?
grep -A2 "phase clocks" $O/clk.err | tail -3

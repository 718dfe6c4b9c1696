#!/bin/bash
# A/B of the XCD-aware conv tile order: bench values at VTF_CONV_GROUP_M = 0 (plain) / 4 / 8 / 16
set -o pipefail
B="--no-cpu-baseline --no-extras --sustain-frames 0"
for rep in 1 2; do
for g in 0 4 8 16; do
  for c in c4 c3 c2; do
    VTF_CONV_GROUP_M=$g timeout -k 10 120 python3 bench.py --config $c --steps 10 --warmup 3 $B > gpurun_out/ab_${c}_g${g}_r$rep.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab_${c}_g${g}_r$rep.json'));print('$c g=$g rep $rep', d['value'], d['ms_per_step'])"
  done
done
done

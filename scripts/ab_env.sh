#!/bin/bash
# Interleaved A/B of an environment switch on the bench: bash scripts/ab_env.sh VAR "v1 v2" CONFIG REPS [extra bench args]
set -o pipefail
VAR=$1; VALS=$2; CFG=${3:-c2}; REPS=${4:-3}; shift 4
B="--no-cpu-baseline --no-extras --sustain-frames 0 --steps 30 --warmup 5 $@"
for rep in $(seq 1 $REPS); do
  for v in $VALS; do
    env $VAR=$v timeout -k 10 150 python3 bench.py --config $CFG $B > gpurun_out/ab_tmp.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/ab_tmp.json'));print('$CFG $VAR=$v rep $rep', d['value'], d['ms_per_step'], d['roofline']['avg_launch_ms'])"
  done
done

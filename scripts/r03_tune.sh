#!/bin/bash
# c2 re-tune after the round-3 k_pnet changes, interleaved twice on one box:
# lanes 3 / 4, PNet quota 2 / 4 / 1, chunk 4 / 2.   bash scripts/r03_tune.sh TAG
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/tune_${1:-a}
mkdir -p $O
run() {  # label, env..., -- bench args
  local label=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 $BARGS > $O/c2.json 2> $O/c2.err || exit $?
  python3 -c "import json; d=json.load(open('$O/c2.json')); print('$label c2', d['value'], d['ms_per_step'])"
}
for rep in 1 2; do
  BARGS="--lanes 3" run "lanes3 q2 c4" VTF_PNET_QUOTA=2
  BARGS="--lanes 4" run "lanes4 q2 c4" VTF_PNET_QUOTA=2
  BARGS="--lanes 3" run "lanes3 q4 c4" VTF_PNET_QUOTA=4
  BARGS="--lanes 3" run "lanes3 q1 c4" VTF_PNET_QUOTA=1
  BARGS="--lanes 3" run "lanes3 q4 c2" VTF_PNET_QUOTA=4 VTF_PNET_CHUNK=2
done

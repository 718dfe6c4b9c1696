#!/bin/bash
# default c2 bench (625 det-batches + the 10k-frame sustained leg): 3 lanes vs 4 lanes on 8 HW queues
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05ln2}
mkdir -p $O
for rep in 1 2; do
  for v in 3 4q; do
    case $v in 4q) L=4; E="GPU_MAX_HW_QUEUES=8";; *) L=$v; E="";; esac
    env $E timeout -k 10 400 python3 bench.py --lanes $L --no-cpu-baseline > $O/c2_$v.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2_$v.json')); print('lanes $v', 'c2', d['value'], d['ms_per_step'], 'sustained', d.get('sustained', {}).get('value'), 'host', d.get('host_frames', {}).get('value'))"
  done
done

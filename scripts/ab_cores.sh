#!/bin/bash
# c2 3-lane: default vs FaceNet convs on 15-KB k_conv tiles (co-resident with a running k_pnet)
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/co_${1:-a}
mkdir -p $O
for rep in 1 2; do
  timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err
  python3 -c "import json; d=json.load(open('$O/c2.json')); print('c2 default', d['value'], d['ms_per_step'])"
  VTF_DMA_BF16=0 VTF_CONV_BF16_SMALL=1000 timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err
  python3 -c "import json; d=json.load(open('$O/c2.json')); print('c2 facenet-15KB', d['value'], d['ms_per_step'])"
done

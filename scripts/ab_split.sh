#!/bin/bash
# bf16 split-K policy A/B (VTF_SPLIT_TILES / VTF_SPLIT_WG): FaceNet encoder-only and c2, interleaved
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/spl_${1:-a}
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_facenet_gpu.py > $O/tests.log 2>&1
tail -1 $O/tests.log
for rep in 1 2; do
  for cfg in "192 512" "768 1536" "768 2048"; do
    set -- $cfg
    VTF_SPLIT_TILES=$1 VTF_SPLIT_WG=$2 timeout -k 10 300 python3 bench.py --det-model none --enc-model facenet --steps 40 --no-cpu-baseline --no-extras > $O/fn.json 2> $O/fn.err
    python3 -c "import json; d=json.load(open('$O/fn.json')); print('split $1 $2 facenet', d['value'], d['ms_per_step'])"
  done
done
for rep in 1 2; do
  for cfg in "192 512" "768 1536"; do
    set -- $cfg
    VTF_SPLIT_TILES=$1 VTF_SPLIT_WG=$2 timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('split $1 $2 c2', d['value'], d['ms_per_step'])"
  done
done

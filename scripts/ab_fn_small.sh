#!/bin/bash
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/fs_${1:-a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_facenet_gpu.py tests/test_shapes_gpu.py -k "facenet" > $O/tests.log 2>&1
tail -1 $O/tests.log
for arm in 1 0 1 0; do
  VTF_CONV_DMA=$arm timeout -k 10 300 python3 bench.py --det-model none --enc-model facenet --frame 224 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/fn_$arm.json 2> $O/fn_$arm.err
  python3 -c "import json; d=json.load(open('$O/fn_$arm.json')); print('facenet small=$arm', d['value'], d['ms_per_step'])"
done
VTF_CONV_DMA=1 bash scripts/facenet_layers.sh s1_${1:-a}
VTF_CONV_DMA=0 bash scripts/facenet_layers.sh s0_${1:-a}
head -1 gpurun_out/fn_s1_${1:-a}/layers.txt gpurun_out/fn_s0_${1:-a}/layers.txt
for arm in 1 0; do
  VTF_CONV_DMA=$arm timeout -k 10 300 python3 bench.py --steps 200 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2_$arm.json 2> $O/c2_$arm.err
  python3 -c "import json; d=json.load(open('$O/c2_$arm.json')); print('c2 dma=$arm', d['value'], d['ms_per_step'])"
done

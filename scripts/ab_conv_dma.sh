#!/bin/bash
# LDS-DMA conv: GPU tests of the bf16 users, then A/B (VTF_CONV_DMA=1/0) on the FaceNet
# encoder-only bench and the c2 headline, plus kernel stats
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cd_${1:-a}
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_facenet_gpu.py tests/test_yolo_gpu.py tests/test_rcnn_gpu.py ${TESTS_EXTRA} > $O/tests.log 2>&1
grep -E "passed|failed|error" $O/tests.log | tail -2
for arm in 1 0 1 0; do
  VTF_CONV_DMA=$arm timeout -k 10 300 python3 bench.py --det-model none --enc-model facenet --frame 224 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/fn_$arm.json 2> $O/fn_$arm.err
  python3 -c "import json; d=json.load(open('$O/fn_$arm.json')); print('facenet dma=$arm', d['value'], d['ms_per_step'])"
done
for arm in 1 0; do
  VTF_CONV_DMA=$arm timeout -k 10 300 python3 bench.py --steps 200 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2_$arm.json 2> $O/c2_$arm.err
  python3 -c "import json; d=json.load(open('$O/c2_$arm.json')); print('c2 dma=$arm', d['value'], d['ms_per_step'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --det-model none --enc-model facenet --frame 224 --no-cpu-baseline --no-extras --steps 20 --sustain-frames 0 > $O/fn_prof.json 2> $O/fn_prof.err
python3 scripts/kstats.py $O/prof 30 > $O/fn_kernel_stats.txt 2>&1 && rm -rf $O/prof
head -14 $O/fn_kernel_stats.txt

#!/bin/bash
# split-fp16 conv staging experiment: ViT-L encoder-only (c4) faces/s per VTF_CONV_XDBG value
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/xdbg
# needs a library built with -DVTF_CONV_XDBG=1 (HIPFLAGS in video-to-faces_amd/Makefile)
for v in 0 1 2 3 0; do
    VTF_CONV_XDBG=$v timeout -k 10 200 python3 bench.py --config c4 --steps 8 --warmup 2 --no-cpu-baseline > gpurun_out/xdbg/c4_$v.json 2> gpurun_out/xdbg/c4_$v.err
    python3 -c "import json; d=json.load(open('gpurun_out/xdbg/c4_$v.json')); print('xdbg $v', d['value'], d['ms_per_step'])"
done

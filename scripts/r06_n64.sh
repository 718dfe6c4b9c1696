#!/bin/bash
# FaceNet: conv_dma 256 x 64 tiles for Cout = 192 (no half-empty 128-column tile), A/B by forward time
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6n64_${1:-a}
mkdir -p $O
timeout -k 10 300 python3 -u scripts/r06_b17ws.py 20 "VTF_DMA_N64=0,VTF_DMA_N64=1,VTF_B17_SPLIT=0,VTF_B17_SPLIT=0+VTF_DMA_N64=1" facenet > $O/ab.txt 2> $O/ab.err || exit $?
cat $O/ab.txt

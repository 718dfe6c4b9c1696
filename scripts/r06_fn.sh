#!/bin/bash
# FaceNet: Block17 weight row-stride A/B (embeddings compared bitwise), then the per-launch listing
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6fn_${1:-a}
mkdir -p $O
timeout -k 10 300 python3 -u scripts/r06_b17ws.py 20 "${2:-VTF_B17_WS=896,VTF_B17_WS=960,VTF_B17_WS=928,VTF_B17_WS=1008}" > $O/ws.txt 2> $O/ws.err || exit $?
cat $O/ws.txt
bash scripts/facenet_layers.sh r6fn_${1:-a}_layers > /dev/null 2>&1 || exit $?

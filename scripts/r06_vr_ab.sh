#!/bin/bash
# k_pnet vertical reuse: MTCNN parity tests with VTF_PNET_VR=1, then k_pnet solo times (probe_pnet
# child, events) interleaved VR off / on and chunk x quota variants, then c2 (300 det-batches).
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6vr_${1:-a}
mkdir -p $O
VTF_PNET_VR=1 timeout -k 10 600 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_mtcnn_gpu.py tests/test_shapes_gpu.py -k "mtcnn or pnet or nms" > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/tests.log | tail -2; grep -E "^FAILED|stage-1 cell" $O/tests.log | head
[ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  for cfg in "0 4 2" "1 4 2" "1 8 1" "1 16 1"; do
    set -- $cfg
    VTF_PNET_VR=$1 VTF_PNET_CHUNK=$2 VTF_PNET_QUOTA=$3 timeout -k 10 120 python3 -u scripts/probe_pnet.py child > $O/p.txt 2> $O/p.err || exit $?
    echo "vr $1 chunk $2 quota $3 $(tail -1 $O/p.txt)"
  done
done
for rep in 1 2; do
  for cfg in "0 4 2" "1 4 2" "1 8 1"; do
    set -- $cfg
    VTF_PNET_VR=$1 VTF_PNET_CHUNK=$2 VTF_PNET_QUOTA=$3 timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras --sustain-frames 0 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('vr $1 chunk $2 quota $3 c2', d['value'], d['ms_per_step'], d['faces_per_frame'])"
  done
done

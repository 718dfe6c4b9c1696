#!/bin/bash
# FaceNet stem head (blob + conv2d_1a fused), vectorised blob / maxpool: GPU tests, per-layer trace,
# then c4-FaceNet and c2 A/B against the HEAD build (lib/libvtf_hip_base.so), interleaved
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/${1:-r05st}
mkdir -p $O
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_facenet_gpu.py tests/test_shapes_gpu.py -k "facenet or stem or blob or encode or c3 or chain" > $O/tests.log 2>&1
rc=$?; tail -3 $O/tests.log; grep -E "stem head|fused vs" $O/tests.log | head; [ $rc -eq 0 ] || exit $rc
bash scripts/facenet_layers.sh r05st bf16 && head -12 gpurun_out/fn_r05st/layers.txt && tail -22 gpurun_out/fn_r05st/layers.txt
B="--no-cpu-baseline --no-extras --sustain-frames 0"
for rep in 1 2; do
  for v in base new; do
    [ $v = base ] && E="VTF_HIP_LIB=$GRAFT_REPO_ROOT/video-to-faces_amd/lib/libvtf_hip_base.so" || E=""
    env $E timeout -k 10 300 python3 bench.py --config c4 --enc-model facenet --steps 40 $B > $O/c4.json 2> $O/c4.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c4.json')); print('$v', 'c4-facenet', d['value'], d['ms_per_step'])"
    env $E timeout -k 10 300 python3 bench.py --steps 300 $B > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$v', 'c2', d['value'], d['ms_per_step'])"
  done
done

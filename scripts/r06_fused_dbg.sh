#!/bin/bash
# which change moves test_fused_candidate_nets_match_layer_path: base / sort-only / max4-only / both
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6fd_${1:-a}
mkdir -p $O
for v in base sort max4 ""; do
  lib=$PWD/video-to-faces_amd/lib/libvtf_hip${v:+_$v}.so
  VTF_HIP_LIB=$lib timeout -k 10 200 python -u -m pytest -v --timeout 100 --timeout-method thread -m gpu tests/test_mtcnn_gpu.py -k "fused_candidate or span_convs" > $O/t_$v.log 2>&1
  echo "lib ${v:-new}: $(grep -cE 'PASSED' $O/t_$v.log) passed, $(grep -cE 'FAILED' $O/t_$v.log) failed; $(grep -E '^E  +At index|^E  +assert' $O/t_$v.log | head -2 | tr '\n' ' ')"
done

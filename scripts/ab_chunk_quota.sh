#!/bin/bash
# k_pnet chunk x quota at 8 tiles per workgroup (full default bench), interleaved twice
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/cq_${1:-a}
mkdir -p $O
VTF_PNET_CHUNK=1 VTF_PNET_QUOTA=8 timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_mtcnn_gpu.py -k "720p or small or shapes" > $O/tests.log 2>&1
echo "chunk 1 tests: $(tail -1 $O/tests.log)"
for rep in 1 2; do
  for cfg in "2 4" "1 8" "4 2"; do
    set -- $cfg
    VTF_PNET_CHUNK=$1 VTF_PNET_QUOTA=$2 timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-extras > $O/c2.json 2> $O/c2.err
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('chunk=$1 quota=$2 c2', d['value'], d['ms_per_step'])"
  done
done

#!/bin/bash
# k_pnet conv2 split-output stores through a cross-half lane exchange (C2_XCH): GPU suite, LDS conflicts, same-box A/B vs
# the previous library (lib/libvtf_hip_base.so): k_pnet pair solo + c2 300 det-batches, interleaved
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6xch_${1:-a}
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu tests > $O/gpu_tests.log 2>&1 || { tail -30 $O/gpu_tests.log; exit 1; }
grep -E "passed|failed" $O/gpu_tests.log | tail -1
bash scripts/r06_pnet_ldsconf.sh xch_${1:-a} "16" || exit $?
B=$PWD/video-to-faces_amd/lib/libvtf_hip_base.so
N=$PWD/video-to-faces_amd/lib/libvtf_hip.so
for rep in 1 2 3; do
  for lib in $B $N; do
    VTF_HIP_LIB=$lib timeout -k 10 120 python3 -u scripts/probe_pnet.py child > $O/p.txt 2> $O/p.err || exit $?
    echo "$(basename $lib) pnet $(tail -1 $O/p.txt)"
    VTF_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$(basename $lib) c2', d['value'], d['ms_per_step'], d['faces_per_frame'])"
  done
done

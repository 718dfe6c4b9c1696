#!/bin/bash
# full GPU suite on HEAD, then k_pnet solo + c2 (300 det-batches, distinct frames) vs the round-5 library
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6g_${1:-a}
mkdir -p $O
timeout -k 10 1000 python -u -m pytest -v -rA --timeout 300 --timeout-method thread -m gpu tests > $O/tests.log 2>&1
rc=$?
grep -E "passed|failed|error" $O/tests.log | tail -2; grep -E "^FAILED|c4 chain|stage-1 cell" $O/tests.log | head
[ $rc -eq 0 ] || exit $rc
B=$PWD/video-to-faces_amd/lib/libvtf_hip_base.so
N=$PWD/video-to-faces_amd/lib/libvtf_hip.so
for rep in 1 2; do
  for lib in $B $N; do
    VTF_HIP_LIB=$lib timeout -k 10 120 python3 -u scripts/probe_pnet.py child > $O/p.txt 2> $O/p.err || exit $?
    echo "$(basename $lib) pnet $(tail -1 $O/p.txt)"
    VTF_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 300 --no-cpu-baseline --no-extras > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$(basename $lib) c2', d['value'], d['ms_per_step'], d['faces_per_frame'])"
  done
done

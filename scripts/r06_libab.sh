#!/bin/bash
# same-box A/B: the round-5 library (lib/libvtf_hip_base.so) vs HEAD, c2 300 det-batches on the
# cycled 32-frame pool and on distinct device frames, interleaved; k_pnet solo per library
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6lib_${1:-a}
mkdir -p $O
B=$PWD/video-to-faces_amd/lib/libvtf_hip_base.so
N=$PWD/video-to-faces_amd/lib/libvtf_hip.so
for rep in 1 2; do
  for lib in $B $N; do
    VTF_HIP_LIB=$lib timeout -k 10 120 python3 -u scripts/probe_pnet.py child > $O/p.txt 2> $O/p.err || exit $?
    echo "$(basename $lib) pnet $(tail -1 $O/p.txt)"
    for pool in 32 0; do
      VTF_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 300 --pool $pool --no-cpu-baseline --no-extras > $O/c2.json 2> $O/c2.err || exit $?
      python3 -c "import json; d=json.load(open('$O/c2.json')); print('$(basename $lib) pool $pool c2', d['value'], d['ms_per_step'], d['faces_per_frame'])"
    done
  done
done

#!/bin/bash
# tile sort A/B on c2 windows: 6 interleaved pairs of 20 det-batches, 2 pairs of the default 625
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6sort2_${1:-a}
mkdir -p $O
B=$PWD/video-to-faces_amd/lib/libvtf_hip_base.so
N=$PWD/video-to-faces_amd/lib/libvtf_hip.so
for rep in 1 2 3 4 5 6; do
  for lib in $B $N; do
    VTF_HIP_LIB=$lib timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$(basename $lib) c2 20', d['value'], d['ms_per_step'])"
  done
done
for rep in 1 2; do
  for lib in $B $N; do
    VTF_HIP_LIB=$lib timeout -k 10 400 python3 bench.py --no-cpu-baseline --no-extras --sustain-frames 10000 > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('$(basename $lib) c2 625', d['value'], d['ms_per_step'], d['steps'])"
  done
done

#!/bin/bash
# k_pnet quota 1 vs 2 (chunk 4): pair solo time (probe_pnet) and c2 20-det-batch windows, interleaved
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6q_${1:-a}
mkdir -p $O
for rep in 1 2 3; do
  for q in 2 1; do
    VTF_PNET_QUOTA=$q timeout -k 10 120 python3 -u scripts/probe_pnet.py child > $O/p.txt 2> $O/p.err || exit $?
    echo "quota $q pnet $(tail -1 $O/p.txt)"
  done
done
for rep in 1 2 3 4; do
  for q in 2 1; do
    VTF_PNET_QUOTA=$q timeout -k 10 300 python3 bench.py --steps 20 --warmup 3 --no-cpu-baseline --no-extras > $O/c2.json 2> $O/c2.err || exit $?
    python3 -c "import json; d=json.load(open('$O/c2.json')); print('quota $q c2 20', d['value'], d['ms_per_step'])"
  done
done

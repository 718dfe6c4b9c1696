#!/bin/bash
# k_pnet solo time (probe_pnet child) under several env settings, one line each:
# bash scripts/pnet_env_sweep.sh TAG "VAR=a VAR2=b" "VAR=c" ...
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/pe_${1:-a}
shift
mkdir -p $O
for e in "$@"; do
  env $e timeout -k 10 120 python3 -u scripts/probe_pnet.py child > $O/run.txt 2> $O/run.err
  echo "$e -> $(tail -1 $O/run.txt)"
done

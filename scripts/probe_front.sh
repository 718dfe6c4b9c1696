#!/bin/bash
# kernel stats of one MTCNN det-batch probe (stage counts printed by probe_mtcnn.py)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/front_${1:-0} -o run -- python3 scripts/probe_mtcnn.py 16 5 > gpurun_out/front_${1:-0}.txt 2>&1

#!/bin/bash
# Block35 tail fused into the branches launch: FaceNet GPU tests, then A/B (embeddings bitwise)
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6b35t_${1:-a}
mkdir -p $O
timeout -k 10 400 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/test_facenet_gpu.py > $O/tests.log 2>&1 || { grep -E "^E |FAILED" $O/tests.log | head -20; exit 1; }
grep -E "passed|failed" $O/tests.log | tail -1
timeout -k 10 300 python3 -u scripts/r06_b17ws.py 20 "VTF_B35_TAIL=0,VTF_B35_TAIL=1" facenet > $O/ab.txt 2> $O/ab.err || exit $?
cat $O/ab.txt
timeout -k 10 200 rocprofv3 --kernel-trace -d $O/t -o run -- python3 -u scripts/r06_b17ws.py 3 "VTF_B35_TAIL=1" facenet > /dev/null 2> $O/t.err || exit $?
python3 scripts/kstats.py $O/t 30 | grep -E "block35|conv64|kernel" | cut -c1-100
find $O -name '*.db' -delete

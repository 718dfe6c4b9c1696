#!/bin/bash
# operand row-stride padding A/B: FaceNet Block17 weight stride sweep, ViT-L pre-split GEMM B / A
# padding (event times + bitwise embeddings), then per-kernel stats of k_gemm_x3 per A-pad mode
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6gp_${1:-a}
mkdir -p $O
timeout -k 10 200 python3 -u scripts/r06_b17ws.py 20 "VTF_B17_WS=896,VTF_B17_WS=904,VTF_B17_WS=912,VTF_B17_WS=928,VTF_B17_WS=944,VTF_B17_WS=1000,VTF_B17_WS=1008" facenet > $O/b17.txt 2> $O/b17.err || exit $?
cat $O/b17.txt
timeout -k 10 300 python3 -u scripts/r06_b17ws.py 3 "VTF_GEMM_BPAD=0,VTF_GEMM_BPAD=64,VTF_GEMM_BPAD=128,VTF_GEMM_BPAD=256,VTF_GEMM_BPAD=512" vit_l > $O/vitb.txt 2> $O/vitb.err || exit $?
cat $O/vitb.txt
for ap in 0 64 128 256; do
  VTF_GEMM_APAD=$ap timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/pa$ap -o run -- python3 -u scripts/r06_b17ws.py 3 "VTF_GEMM_BPAD=0" vit_l > $O/pa$ap.txt 2> $O/pa$ap.err || exit $?
  python3 - "$O/pa$ap" "$ap" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)
rows = list(csv.DictReader(open(f[0]))) if f else []
for r in rows:
    if 'k_gemm_x3' in r['Name']:
        print('apad', sys.argv[2], r['Name'][:40], 'calls', r['Calls'], 'avg_us %.2f' % (float(r['AverageNs']) / 1e3), 'total_ms %.2f' % (float(r['TotalDurationNs']) / 1e6))
PY
done
find $O -name '*.db' -delete

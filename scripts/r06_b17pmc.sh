#!/bin/bash
# FaceNet forward under PMC passes (SQ set; TCC hit / miss): k_block17 vs the other FaceNet kernels
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
O=gpurun_out/r6b17p_${1:-a}
mkdir -p $O
SQ="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
timeout -s KILL 120 rocprofv3 --pmc $SQ --kernel-trace --output-format csv -d $O/sq -o run -- python3 -u scripts/r06_b17ws.py 3 "VTF_B17_SPLIT=0" facenet > /dev/null 2> $O/sq.err || exit $?
timeout -s KILL 120 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum --kernel-trace --output-format csv -d $O/tcc -o run -- python3 -u scripts/r06_b17ws.py 3 "VTF_B17_SPLIT=0" facenet > /dev/null 2> $O/tcc.err || exit $?
python3 - $O <<'PY'
import csv, glob, sys, collections
O = sys.argv[1]
def load(d):
    f = glob.glob(O + '/' + d + '/**/*counter_collection.csv', recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(float))
    cnt = collections.Counter()
    for r in csv.DictReader(open(f[0])):
        n = r['Kernel_Name'].split('(')[0][-40:]
        agg[n][r['Counter_Name']] += float(r['Counter_Value'])
        if r['Counter_Name'] == list(agg[n].keys())[0]:
            cnt[n] += 1
    return agg, cnt
sq, c1 = load('sq')
tc, c2 = load('tcc')
for n in sorted(sq, key=lambda k: -sq[k].get('SQ_BUSY_CYCLES', 0))[:12]:
    a = sq[n]; t = tc.get(n, {})
    wc = a.get('SQ_WAVE_CYCLES', 1)
    hit = t.get('TCC_HIT_sum', 0); miss = t.get('TCC_MISS_sum', 0)
    print('%-40s mfma-busy/gui %.3f wait %.2f waitinst %.2f active %.2f ldsconf %.2f  L2 hit %.3f (hit %.3g miss %.3g)' % (
        n, a.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / max(1, a.get('GRBM_GUI_ACTIVE', 1)) / 1024 * 8,
        a.get('SQ_WAIT_ANY', 0) / wc, a.get('SQ_WAIT_INST_ANY', 0) / wc, a.get('SQ_ACTIVE_INST_ANY', 0) / wc,
        a.get('SQ_LDS_BANK_CONFLICT', 0) / max(1, a.get('SQ_LDS_IDX_ACTIVE', 1)), hit / max(1, hit + miss), hit, miss))
PY
find $O -name '*.csv' -size +5M -delete

"""Per-mask k_pnet counter table from scripts/probe_pnet_pmc.sh: python probe_pnet_table.py DIR masks...

Counters are averaged per k_pnet dispatch and divided by the wave count where they are per-wave
sums (instructions), so the table reads as instructions per wave per launch."""
import csv
import glob
import os
import sys
from collections import defaultdict


KF = os.environ.get('KFILTER', '')  # e.g. 'true>' for the exact-levels variant only


def load(d):
    f = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    acc, calls = defaultdict(float), set()
    if not f:
        return acc, 0
    for r in csv.DictReader(open(f[0])):
        if 'k_pnet' not in r['Kernel_Name'] or KF not in r['Kernel_Name']:
            continue
        acc[r['Counter_Name']] += float(r['Counter_Value'])
        calls.add(r.get('Dispatch_Id') or r.get('Correlation_Id'))
    n = max(1, len(calls))
    return {k: v / n for k, v in acc.items()}, n


def main():
    root, masks = sys.argv[1], sys.argv[2:]
    cols = ['SQ_WAVE_CYCLES', 'SQ_WAIT_ANY', 'SQ_ACTIVE_INST_ANY', 'SQ_WAIT_INST_ANY', 'SQ_WAIT_INST_LDS',
            'SQ_LDS_IDX_ACTIVE', 'SQ_LDS_BANK_CONFLICT', 'SQ_VALU_MFMA_BUSY_CYCLES', 'SQ_INSTS_VALU',
            'SQ_INSTS_LDS', 'SQ_INSTS_SALU', 'SQ_INSTS_SMEM', 'SQ_INSTS_VMEM_RD', 'SQ_INSTS_VMEM_WR',
            'GRBM_GUI_ACTIVE', 'SQ_INSTS_BRANCH', 'SQ_WAVES']
    print('per k_pnet dispatch (sums over all waves; divide by waves for per-wave figures)')
    print('%-26s' % 'counter' + ''.join('%14s' % ('mask ' + m) for m in masks))
    data = {}
    for m in masks:
        a, _ = load(os.path.join(root, 'p1_' + m))
        b, _ = load(os.path.join(root, 'p2_' + m))
        c, _ = load(os.path.join(root, 'p3_' + m))
        data[m] = {**a, **b, **c}
    for c in cols:
        print('%-26s' % c + ''.join('%14.4g' % data[m].get(c, float('nan')) for m in masks))


if __name__ == '__main__':
    main()

"""Per-kernel PMC table from the rocprofv3 csv passes of scripts/profile_r02.sh.

  python scripts/pmc_table.py gpurun_out/prof_TAG c2 [top]

For every kernel family (name up to the template arguments kept): calls, average duration
(from the SQ pass's kernel trace), MFMA busy % (SQ_VALU_MFMA_BUSY_CYCLES / (SQ_BUSY_CYCLES*4?):
reported raw and as a fraction of GRBM_GUI_ACTIVE cycles x 4 SIMDs x CUs is not attempted --
we print MFMA-busy per CU-cycle: MFMA_BUSY / (GRBM_GUI_ACTIVE / 8 XCDs * 256 CUs)), wave-parked
(SQ_WAIT_ANY / SQ_WAVE_CYCLES), LDS bank-conflict share (SQ_LDS_BANK_CONFLICT /
SQ_LDS_IDX_ACTIVE), HBM bytes per launch (FETCH_SIZE x 2 gfx950 correction + WRITE_SIZE).
"""
import csv
import glob
import os
import re
import sys
from collections import defaultdict


def load(d):
    f = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)
    if not f:
        return {}
    acc = defaultdict(lambda: defaultdict(float))
    calls = defaultdict(set)
    for r in csv.DictReader(open(f[0])):
        name = re.sub(r'\(anonymous namespace\)::', '', r['Kernel_Name'])
        name = re.sub(r'\(.*', '', name)
        name = re.sub(r'^void ', '', name)
        acc[name][r['Counter_Name']] += float(r['Counter_Value'])
        calls[name].add(r.get('Dispatch_Id') or r.get('Correlation_Id'))
    return {k: (len(calls[k]), v) for k, v in acc.items()}


def durations(d):
    import sqlite3
    f = glob.glob(os.path.join(d, '**', '*results.db'), recursive=True)
    if not f:
        return {}
    c = sqlite3.connect(f[0])
    out = {}
    for n, k, s in c.execute('select name, count(*), sum(duration) from kernels group by name'):
        n = re.sub(r'^void ', '', re.sub(r'\(.*', '', re.sub(r'\(anonymous namespace\)::', '', n)))
        out[n] = (k, s / 1e3)
    return out


def main():
    root, cfg = sys.argv[1], sys.argv[2]
    top = int(sys.argv[3]) if len(sys.argv) > 3 else 14
    sq = load(os.path.join(root, cfg + '_pmc_sq'))
    fe = load(os.path.join(root, cfg + '_pmc_fetch'))
    wr = load(os.path.join(root, cfg + '_pmc_write'))
    tr = durations(os.path.join(root, cfg + '_trace1'))
    names = sorted(tr, key=lambda n: -tr[n][1])[:top]
    print('%-58s %5s %9s %7s %7s %7s %7s %11s %11s' % ('kernel (1-lane trace)', 'calls', 'avg_us', 'mfma%',
                                                      'parked', 'ldsconf', 'valu%', 'fetch_MB', 'write_MB'))
    for n in names:
        k, tot = tr[n]
        row = ['%-58s %5d %9.1f' % (n[:58], k, tot / k)]
        s = sq.get(n)
        if s:
            ks, c = s
            cu_cycles = c.get('GRBM_GUI_ACTIVE', 0) / 8 * 256  # per-XCD GUI cycles summed over 8 XCDs
            mf = c.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / max(1.0, cu_cycles * 4) * 100
            wc = c.get('SQ_WAVE_CYCLES', 0)
            parked = c.get('SQ_WAIT_ANY', 0) / max(1.0, wc) * 100
            act = c.get('SQ_ACTIVE_INST_ANY', 0) / max(1.0, wc) * 100
            lc = c.get('SQ_LDS_BANK_CONFLICT', 0) / max(1.0, c.get('SQ_LDS_IDX_ACTIVE', 0)) * 100
            row.append('%7.1f %7.1f %7.1f %7.1f' % (mf, parked, lc, act))
        else:
            row.append('%7s %7s %7s %7s' % ('-', '-', '-', '-'))
        f = fe.get(n)
        w = wr.get(n)
        row.append('%11.1f' % (2 * f[1]['FETCH_SIZE'] * 1024 / f[0] / 1e6) if f else '%11s' % '-')
        row.append('%11.1f' % (w[1]['WRITE_SIZE'] * 1024 / w[0] / 1e6) if w else '%11s' % '-')
        print(' '.join(row))
    print('mfma%: SQ_VALU_MFMA_BUSY_CYCLES / (4 SIMDs x 256 CUs x GRBM_GUI_ACTIVE/8); parked: SQ_WAIT_ANY / '
          'SQ_WAVE_CYCLES; ldsconf: SQ_LDS_BANK_CONFLICT / SQ_LDS_IDX_ACTIVE; valu%: SQ_ACTIVE_INST_ANY / '
          'SQ_WAVE_CYCLES; fetch_MB: FETCH_SIZE (KB) x 2 (gfx950) per launch; write_MB: WRITE_SIZE per launch')


if __name__ == '__main__':
    main()

"""Per-kernel average of a rocprofv3 PMC counter (csv output): python pmc_summary.py DIR [kernel-substring]."""
import csv, glob, os, re, sys
from collections import defaultdict
d = sys.argv[1]
sub = sys.argv[2] if len(sys.argv) > 2 else ''
f = glob.glob(os.path.join(d, '**', '*counter_collection.csv'), recursive=True)[0]
acc = defaultdict(lambda: [0, 0.0])
for r in csv.DictReader(open(f)):
    name = re.sub(r'\(.*', '', r['Kernel_Name'])
    if sub and sub not in name:
        continue
    key = (name, r['Counter_Name'])
    acc[key][0] += 1
    acc[key][1] += float(r['Counter_Value'])
for (n, c), (k, v) in sorted(acc.items(), key=lambda x: -x[1][1])[:30]:
    print('%-60s %-12s calls %5d  avg %.4g  total %.4g' % (n[:60], c, k, v / k, v))

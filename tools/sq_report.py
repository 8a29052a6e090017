"""Per-wave SQ counter means per kernel from a rocprofv3 --pmc csv directory."""
import csv, glob, sys
from collections import defaultdict
d, tag = sys.argv[1], sys.argv[2]
flt = sys.argv[3] if len(sys.argv) > 3 else 'jpeg'
tot = defaultdict(lambda: defaultdict(float))
for f in glob.glob(d + '/**/*counter_collection.csv', recursive=True):
    for r in csv.DictReader(open(f)):
        k = r['Kernel_Name'][:40]
        tot[k][r['Counter_Name']] += float(r['Counter_Value'])
for k, c in tot.items():
    if flt not in k: continue
    w = c.get('SQ_WAVES', 1) or 1
    print(tag, k, ' '.join(f"{n[3:]}={v / w:.0f}" for n, v in sorted(c.items()) if n != 'SQ_WAVES'), 'waves', int(w))

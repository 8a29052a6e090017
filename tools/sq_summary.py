"""Summarise tools/sq_counters.sh output: per-kernel mean counters per launch."""
import collections, csv, sys
d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for p in ('p1', 'p2'):
    for r in csv.DictReader(open(f'{d}/{p}/run_counter_collection.csv')):
        agg[r['Kernel_Name'].split('(')[0]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, c in agg.items():
    if 'jpeg' not in k and 'rrc' not in k:
        continue
    m = {n: sum(v) / len(v) for n, v in c.items()}
    w = m.get('SQ_WAVES', 1)
    print(k, 'waves', w)
    for n in sorted(m):
        print(f'   {n:24s} {m[n]:14.0f}  per-wave {m[n] / w:10.1f}')

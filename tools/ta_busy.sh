#!/bin/bash
# Texture-address (TA) and GPU-active counters for K1 alone and K2 alone
# (one --pmc pass each): tools/ta_busy.sh <tag>
export TMPDIR=/tmp
OUT=gpurun_out/${1:-ta}; mkdir -p $OUT
for o in 1 4; do
  timeout -s KILL 120 rocprofv3 --pmc TA_BUSY_avr TA_BUSY_max GRBM_GUI_ACTIVE GRBM_COUNT --output-format csv -d $OUT/o$o -o run -- python3 bench.py --steps 48 --warmup 12 --no-cpu-baseline --no-host-check --only $o > $OUT/o$o.log 2>&1 || exit 1
done
python3 - $OUT <<'PY'
import collections, csv, sys
d = sys.argv[1]
for o in ('o1', 'o4'):
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for r in csv.DictReader(open(f'{d}/{o}/run_counter_collection.csv')):
        agg[r['Kernel_Name'].split('(')[0]][r['Counter_Name']].append(float(r['Counter_Value']))
    for k, c in agg.items():
        if 'jpeg' in k:
            m = {n: sum(v) / len(v) for n, v in c.items()}
            print(o, k, {n: round(v) for n, v in m.items()},
                  'TA_busy/GUI_active(per XCD)', round(m.get('TA_BUSY_avr', 0) / (m.get('GRBM_GUI_ACTIVE', 1) / 8), 3))
PY

#!/bin/bash
# SQ instruction counts of K2's timed launches with and without its parts
# (timing-only flags skip work): tools/k2_valu.sh <tag>
export TMPDIR=/tmp
OUT=gpurun_out/${1:-k2valu}; mkdir -p $OUT
for f in 0 1792 512 256; do
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/f$f -o run -- python3 bench.py --steps 48 --warmup 12 --no-cpu-baseline --no-host-check --only 4 --k2flags $f > $OUT/f$f.log 2>&1 || exit 1
done
python3 - $OUT <<'PY'
import collections, csv, sys
d = sys.argv[1]
for f in (0, 1792, 512, 256):
    rows = collections.defaultdict(dict)
    for r in csv.DictReader(open(f'{d}/f{f}/run_counter_collection.csv')):
        if 'color_resize' in r['Kernel_Name']:
            rows[int(r['Dispatch_Id'])][r['Counter_Name']] = float(r['Counter_Value'])
    last = [rows[k] for k in sorted(rows)[-4:]]  # the 4 timed launches (12 batches x 512)
    m = {n: sum(x[n] for x in last) / len(last) / 6144 for n in last[0]}
    print('k2flags', f, {n: round(v) for n, v in sorted(m.items())})
PY

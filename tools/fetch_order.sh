#!/bin/bash
# K1's FETCH_SIZE with and without the size-grouped workgroup order
# (K1 fetch rose 16% from r3d to r3e, the order being the only
# kept K1 change in between).   tools/fetch_order.sh <tag>
TAG=${1:-ord}
mkdir -p gpurun_out
export TMPDIR=/tmp
for o in 1 0; do
  FFCV_K1_ORDER=$o timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/${TAG}_k1o$o -o run -- python3 bench.py --steps 48 --warmup 24 --no-cpu-baseline --uniform-launches --no-host-check --no-later-epochs --no-c5 --parity-rows 0 > gpurun_out/${TAG}_k1o$o.log 2>&1 || exit 1
  python3 - <<PY
import csv, collections
v = collections.defaultdict(list)
for r in csv.DictReader(open('gpurun_out/${TAG}_k1o$o/run_counter_collection.csv')):
    if r['Counter_Name'] == 'FETCH_SIZE':
        v[r['Kernel_Name'].split('(')[0]].append(float(r['Counter_Value']))
for k, x in v.items():
    if 'jpeg' in k:
        print('K1_ORDER=$o', k, 'launches', len(x), 'FETCH KB per 12288-image launch %.0f' % (sum(x) / len(x)), 'per image %.1f KB' % (sum(x) / len(x) / 12288))
PY
done

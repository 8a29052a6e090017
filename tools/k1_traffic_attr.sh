#!/bin/bash
# K1's HBM traffic by phase: FETCH_SIZE and WRITE_SIZE,
# one PMC pass each, over K1-only launches of 12,288 images for timing-only
# builds that stop after a phase (build/ab/<name>.so from
# tools/build_variant.sh: stop8 -DK1_STOP=8 gather + draws + header + parse +
# arena, stop1 + tables, stop2 + de-stuff, stop4 + sync rounds, nozero the
# full kernel without the window zeroing) and the full build.
#   tools/k1_traffic_attr.sh <tag> ["variants"]
TAG=${1:-k1t}
VARS=${2:-"stop8 stop1 stop2 stop4 nozero full"}
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python3 -c "import bench; bench.make_unique('jpg', 256, 65536, 0, 16)" || exit 1
for v in $VARS; do
  lib="--lib build/ab/$v.so"; [ $v = full ] && lib=""
  for c in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv -d gpurun_out/${TAG}_${v}_$c -o run -- python3 bench.py $lib --only 1 --steps 48 --warmup 24 --no-cpu-baseline --uniform-launches --no-host-check --no-later-epochs --no-c5 --parity-rows 0 --no-kernel-events > gpurun_out/${TAG}_${v}_$c.log 2>&1 || { tail -3 gpurun_out/${TAG}_${v}_$c.log; exit 1; }
    python3 - <<PY
import csv, collections
d = collections.defaultdict(float)
for r in csv.DictReader(open('gpurun_out/${TAG}_${v}_$c/run_counter_collection.csv')):
    if 'entropy' in r['Kernel_Name'] and r['Counter_Name'] == '$c':
        d[r['Dispatch_Id']] += float(r['Counter_Value'])
x = [d[k] for k in sorted(d, key=int)][-2:]  # the two timed K1-only launches (12,288 images each)
print('$v $c bytes per image %.0f' % (sum(x) / len(x) * 1024 / 12288), 'launches', len(d))
PY
  done
done
echo ATTR_DONE

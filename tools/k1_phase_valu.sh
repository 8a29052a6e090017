#!/bin/bash
# K1's VALU per image by phase: timing-only builds that end K1 after a phase
# (-DK1_STOP=2 de-stuff, 4 sync pass, 5 write pass; build/ab/stop<N>.so from
# tools/build_variant.sh) and the full build, one SQ pass each over
# K1-only launches of 12,288 images.   tools/k1_phase_valu.sh <tag> ["variants"]
# (variants: build/ab/<name>.so, or full = the working tree)
TAG=${1:-k1v}
VARS=${2:-"stop2 stop4 stop5 full"}
mkdir -p gpurun_out
export TMPDIR=/tmp
# generate (and cache in /tmp) the samples outside the profiler: a worker pool
# forked under rocprofv3 hung at its end on a fresh box
timeout -k 10 600 python3 -c "import bench; bench.make_unique('jpg', 256, 65536, 0, 16)" || exit 1
for v in $VARS; do
  lib="--lib build/ab/$v.so"; [ $v = full ] && lib=""
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY --output-format csv -d gpurun_out/${TAG}_$v -o run -- python3 bench.py $lib --only 1 --steps 48 --warmup 24 --no-cpu-baseline --uniform-launches --no-host-check --no-later-epochs --no-c5 --parity-rows 0 --no-kernel-events > gpurun_out/${TAG}_$v.log 2>&1 || { tail -3 gpurun_out/${TAG}_$v.log; exit 1; }
  python3 - <<PY
import csv, collections
v = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.Counter()
for r in csv.DictReader(open('gpurun_out/${TAG}_$v/run_counter_collection.csv')):
    k = r['Kernel_Name'].split('(')[0]
    if 'entropy' not in k: continue
    v[r['Counter_Name']][r['Dispatch_Id']] += float(r['Counter_Value'])
for c, d in v.items():
    x = list(d.values())
    print('$v', c, 'per image %.0f' % (sum(x) / len(x) / 12288), 'launches', len(x))
PY
done

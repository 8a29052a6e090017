#!/bin/bash
# C5 (raw RRC 448) instruction / time split by diagnostic stop builds
# (-DRRC_STOP=n: 1 set-up only, 2 + staging, 3 + the linear walk's column taps,
# 4 + the area walk's column taps):
#   tools/c5_parts.sh <tag> "new rrcstop1 rrcstop2 rrcstop3"
# one rocprofv3 SQ pass (+ kernel trace for durations) per build, launches of
# 2,560 images one at a time; prints VALU / SALU / LDS per image and ns per image.
# EXTRA: more bench.py arguments (e.g. EXTRA="--draw-scale 0.79,0.9").
TAG=$1; V=${2:-"new rrcstop1 rrcstop2 rrcstop3"}
export TMPDIR=/tmp
# warm the box first (first import of torch, the /tmp sample cache) with
# output going to a file: a profiled run that is silent for 3 minutes is killed
timeout -k 10 300 python3 bench.py --config c5 --steps 2 --warmup 1 --unique 1024 --no-host-check --no-cpu-baseline --parity-rows 0 --no-kernel-events > gpurun_out/${TAG}_warm.log 2>&1 || { tail -3 gpurun_out/${TAG}_warm.log; exit 1; }
for v in $V; do
  lib=""; [ $v != new ] && lib="--lib build/ab/$v.so"
  d=gpurun_out/${TAG}_$v
  echo "c5_parts: $v $(date +%T)" >> gpurun_out/${TAG}_progress.txt
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d $d -o run -- python3 bench.py $lib --config c5 --steps 40 --warmup 10 --unique 1024 --inflight 1 --no-cpu-baseline --no-host-check --parity-rows 0 --no-kernel-events $EXTRA > $d.log 2>&1 || { tail -3 $d.log; exit 1; }
  python3 - "$d" "$v" <<'PY'
import csv, glob, sys, collections
d, v = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(glob.glob(d + '/**/run_counter_collection.csv', recursive=True)[0])))
acc = collections.defaultdict(lambda: collections.defaultdict(float)); n = collections.defaultdict(set)
for r in rows:
    if 'rrc_raw_kernel' not in r['Kernel_Name']: continue
    acc[r['Counter_Name']]['v'] += float(r['Counter_Value']); n[r['Counter_Name']].add(r['Dispatch_Id'])
st = [r for r in csv.DictReader(open(glob.glob(d + '/**/run_kernel_stats.csv', recursive=True)[0])) if 'rrc_raw_kernel' in r['Name']]
imgs = 2560
k = {c: acc[c]['v'] / len(n[c]) / imgs for c in acc}
print(f"{v:10s} valu/img {k.get('SQ_INSTS_VALU',0):9.0f} salu {k.get('SQ_INSTS_SALU',0):8.0f} lds {k.get('SQ_INSTS_LDS',0):7.0f} vmem {k.get('SQ_INSTS_VMEM',0):6.0f} waves {k.get('SQ_WAVES',0):5.1f} wait {k.get('SQ_WAIT_ANY',0)/max(1,k.get('SQ_WAVE_CYCLES',1)):.3f} waitinst {k.get('SQ_WAIT_INST_ANY',0)/max(1,k.get('SQ_WAVE_CYCLES',1)):.3f} ns/img {float(st[0]['AverageNs'])/imgs:7.1f}")
PY
done

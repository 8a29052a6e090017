#!/bin/bash
# Per-band K2 (jpeg_color_resize_kernel) instructions / time by
# phase: diagnostic stop builds -DK2_STOP=n (1 set-up, 2 + plane tiles,
# 3 + colour pass; tools/build_variant.sh k2stopN -DK2_STOP=N):
#   tools/k2_parts.sh <tag> "new k2stop1 k2stop2 k2stop3"
TAG=$1; V=${2:-"new k2stop1 k2stop2 k2stop3"}
export TMPDIR=/tmp
# warm the box first (first import of torch, the /tmp sample cache) with
# output going to a file: a profiled run that is silent for 3 minutes is killed
timeout -k 10 300 python3 -u bench.py --steps 2 --warmup 1 --no-host-check --no-cpu-baseline --parity-rows 0 --no-kernel-events --no-later-epochs --no-c5 > gpurun_out/${TAG}_warm.log 2>&1 || { tail -3 gpurun_out/${TAG}_warm.log; exit 1; }
for v in $V; do
  lib=""; [ $v != new ] && lib="--lib build/ab/$v.so"
  d=gpurun_out/${TAG}_$v
  echo "k2_parts: $v $(date +%T)" >> gpurun_out/${TAG}_progress.txt
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY --output-format csv -d $d -o run -- python3 bench.py $lib --steps 24 --warmup 24 --uniform-launches --no-cpu-baseline --no-host-check --parity-rows 0 --no-kernel-events --no-later-epochs --no-c5 > $d.log 2>&1 || { tail -3 $d.log; exit 1; }
  python3 - "$d" "$v" <<'PY'
import csv, glob, sys, collections
d, v = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(glob.glob(d + '/**/run_counter_collection.csv', recursive=True)[0])))
st = list(csv.DictReader(open(glob.glob(d + '/**/run_kernel_stats.csv', recursive=True)[0])))
for kn in ('jpeg_color_resize_kernel', 'jpeg_entropy_kernel', 'jpeg_idct_kernel'):
    acc = collections.defaultdict(float); n = collections.defaultdict(set)
    for r in rows:
        if kn not in r['Kernel_Name']: continue
        acc[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']].add(r['Dispatch_Id'])
    imgs = 12288
    k = {c: acc[c] / len(n[c]) / imgs for c in acc}
    ns = [float(x['AverageNs']) / imgs for x in st if kn in x['Name']]
    print(f"{v:9s} {kn[:20]:20s} valu/img {k.get('SQ_INSTS_VALU',0):9.0f} salu {k.get('SQ_INSTS_SALU',0):8.0f} lds {k.get('SQ_INSTS_LDS',0):7.0f} vmem {k.get('SQ_INSTS_VMEM',0):6.0f} wait {k.get('SQ_WAIT_ANY',0)/max(1,k.get('SQ_WAVE_CYCLES',1)):.3f} ns/img {ns[0] if ns else 0:7.1f}")
PY
done

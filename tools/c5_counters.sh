#!/bin/bash
# C5 raw kernel counters by crop-scale band (ratio 1): VALU / LDS / SALU
# instructions and wave cycles per image (images = SQ_WAVES / 112: 28 bands
# of 16 rows x 4 waves per 448-row image), and the kernel's average time.
#   tools/c5_counters.sh <tag> [lib]
TAG=${1:-c5c}; LIB=${2:+--lib $2}
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python3 -u bench.py --config c5 --unique 1024 --steps 2 --warmup 1 --no-cpu-baseline --no-later-epochs --parity-rows 0 > gpurun_out/${TAG}_warm.log 2>&1 || { tail -3 gpurun_out/${TAG}_warm.log; exit 1; }
for b in ${BANDS:-0.60,0.76 0.80,0.86 0.94,1.0}; do
  d=gpurun_out/${TAG}_$b
  timeout -s KILL 240 rocprofv3 --kernel-trace --stats --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_LDS --output-format csv -d $d -o run -- python3 bench.py $LIB --config c5 --unique 1024 --steps 20 --warmup 5 --uniform-launches --inflight 1 --no-cpu-baseline --no-host-check --parity-rows 0 --no-kernel-events --no-later-epochs --draw-scale $b > $d.log 2>&1 || { tail -3 $d.log; exit 1; }
  python3 - "$d" "$b" <<'PY'
import csv, glob, sys, collections
d, b = sys.argv[1], sys.argv[2]
rows = list(csv.DictReader(open(glob.glob(d + '/**/run_counter_collection.csv', recursive=True)[0])))
st = list(csv.DictReader(open(glob.glob(d + '/**/run_kernel_stats.csv', recursive=True)[0])))
acc = collections.defaultdict(float); n = collections.defaultdict(set)
for r in rows:
    if 'rrc_raw_kernel' not in r['Kernel_Name']: continue
    acc[r['Counter_Name']] += float(r['Counter_Value']); n[r['Counter_Name']].add(r['Dispatch_Id'])
k = {c: acc[c] / len(n[c]) for c in acc}
imgs = k['SQ_WAVES'] / 112
per = {c: v / imgs for c, v in k.items()}
ns = [float(x['AverageNs']) for x in st if 'rrc_raw_kernel' in x['Name']]
print(f"scale {b} images/launch {imgs:.0f} valu/img {per['SQ_INSTS_VALU']:.0f} salu {per['SQ_INSTS_SALU']:.0f} lds {per['SQ_INSTS_LDS']:.0f} "
      f"wave_cycles/img {per['SQ_WAVE_CYCLES']:.0f} wait_any {k['SQ_WAIT_ANY']/k['SQ_WAVE_CYCLES']:.3f} wait_lds {k['SQ_WAIT_INST_LDS']/k['SQ_WAVE_CYCLES']:.3f} "
      f"ns/img {ns[0]/imgs if ns else 0:.1f}", flush=True)
PY
done

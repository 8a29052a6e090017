#!/bin/bash
# Per-kernel time of the C3 decode at inflight 1 under K2 diagnostic flags
# (FFCV_K2_FLAGS; bits 3/4 skip work and give wrong output -- timing only).
#   tools/k2_breakdown.sh "0 8 16 24"
export TMPDIR=/tmp
for f in ${1:-0 8 16 24}; do
  OUT=gpurun_out/k2b_$f
  FFCV_K2_FLAGS=$f timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 bench.py --dataset-size 65536 --steps 20 --warmup 3 --no-cpu-baseline --inflight 1 > $OUT.log 2>&1 || exit 1
  python3 - "$OUT" "$f" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if 'jpeg' in r['Name']:
        print('flags', sys.argv[2], r['Name'][:40], 'avg_us', round(float(r['AverageNs']) / 1e3, 1))
PY
done

#!/bin/bash
# Diagnostic pass: K1 phase stamps at 512 and 2048 images, per-kernel time at
# inflight 1 and 8, SQ counters at inflight 8.   tools/diag.sh <tag>
TAG=${1:-d}
mkdir -p gpurun_out
export TMPDIR=/tmp
for b in 512 2048; do
  timeout -k 10 120 python tools/jpeg_phases.py $b > gpurun_out/ph${b}_$TAG.log 2>&1 || exit 1
  grep -v amdgpu.ids gpurun_out/ph${b}_$TAG.log
done
for k in 1 8; do
  OUT=gpurun_out/kt${k}_$TAG
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT -o run -- \
    python3 bench.py --dataset-size 65536 --steps 20 --warmup 3 --no-cpu-baseline --inflight $k > $OUT.log 2>&1 || exit 1
  tail -1 $OUT.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('inflight $k', d['value'])"
  python3 - "$OUT" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    print('  ', r['Name'][:40], 'calls', r['Calls'], 'avg_us', round(float(r['AverageNs']) / 1e3, 1))
PY
done
bash tools/sq_counters.sh $TAG > /dev/null 2>&1 && python tools/sq_summary.py gpurun_out/sq_$TAG

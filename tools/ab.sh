#!/bin/bash
# A/B full C3 bench across library variants: tools/ab.sh "default jw2" [inflight] [extra bench args]
for v in $1; do
  lib=""; [ "$v" != default ] && lib=build/ab/$v.so
  timeout -k 10 200 python bench.py --lib $lib --dataset-size 262144 --steps ${STEPS:-400} --warmup 20 --no-cpu-baseline --inflight ${2:-8} $3 > gpurun_out/ab_$v.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/ab_$v.log').read().strip().splitlines()[-1]);print('$v', 'inflight', ${2:-8}, '$3', d['value'], 'img/s', d['roofline']['kernel_ms'], 'ms/launch')"
done

#!/bin/bash
# Alternating full-C3 A/B of library variants: tools/ab_full.sh "a b" reps [bench args]
for r in $(seq ${2:-3}); do for v in $1; do
  lib=""; [ "$v" != default ] && lib="--lib build/ab/$v.so"
  timeout -k 10 200 python bench.py $lib --no-cpu-baseline --steps 1200 $3 > gpurun_out/abf_${v}.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/abf_${v}.log').read().strip().splitlines()[-1]);print('$v', round(d['value']))"
done; done

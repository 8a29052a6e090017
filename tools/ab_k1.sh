#!/bin/bash
# A/B K1-only and full C3 rates across library variants (build/ab/<name>.so):
#   tools/ab_k1.sh "default jw5 ..."   -> gpurun_out/abk1_<name>_{k1,full}.log + summary lines
for v in $1; do
  lib=""; [ "$v" != default ] && lib="--lib build/ab/$v.so"
  timeout -k 10 200 python bench.py $lib --no-cpu-baseline --only 1 --no-host-check > gpurun_out/abk1_${v}_k1.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py $lib --no-cpu-baseline > gpurun_out/abk1_${v}_full.log 2>&1 || exit 1
  python -c "
import json
k=json.loads(open('gpurun_out/abk1_${v}_k1.log').read().strip().splitlines()[-1])
f=json.loads(open('gpurun_out/abk1_${v}_full.log').read().strip().splitlines()[-1])
print('$v', 'K1', round(k['value']), 'full', round(f['value']))"
done

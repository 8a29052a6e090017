#!/bin/bash
# A/B K2-only and full C3 rates across library variants (build/ab/<name>.so):
#   tools/ab_k2only.sh "default v1 ..."   -> gpurun_out/abk2_<name>_{k2,full}.log + summary lines
for v in $1; do
  lib=""; [ "$v" != default ] && lib="--lib build/ab/$v.so"
  timeout -k 10 200 python bench.py $lib --no-cpu-baseline --only 4 --no-host-check > gpurun_out/abk2_${v}_k2.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py $lib --no-cpu-baseline > gpurun_out/abk2_${v}_full.log 2>&1 || exit 1
  python -c "
import json
k=json.loads(open('gpurun_out/abk2_${v}_k2.log').read().strip().splitlines()[-1])
f=json.loads(open('gpurun_out/abk2_${v}_full.log').read().strip().splitlines()[-1])
print('$v', 'K2', round(k['value']), 'full', round(f['value']))"
done

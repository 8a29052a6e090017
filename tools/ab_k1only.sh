#!/bin/bash
# Alternating K1-alone and full-pipeline rates of library builds:
#   tools/ab_k1only.sh reps "default base ..."   (build/ab/<name>.so; default = in-tree)
for r in $(seq ${1:-2}); do for v in $2; do
  lib=""; [ "$v" != default ] && lib="--lib build/ab/$v.so"
  timeout -k 10 200 python bench.py $lib --no-cpu-baseline --no-later-epochs --only 1 --no-host-check > gpurun_out/ak1_$v.log 2>&1 || exit 1
  timeout -k 10 200 python bench.py $lib --no-cpu-baseline --no-later-epochs > gpurun_out/akf_$v.log 2>&1 || exit 1
  python -c "
import json
k=json.loads(open('gpurun_out/ak1_$v.log').read().strip().splitlines()[-1])
f=json.loads(open('gpurun_out/akf_$v.log').read().strip().splitlines()[-1])
print('$v', 'K1', round(k['value']), 'full', round(f['value']))"
done; done

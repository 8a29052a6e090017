#!/bin/bash
# The driver's bench command alternating over library builds (build/ab/<name>.so; default = in-tree):
#   tools/ab_drv.sh reps "default base"
for r in $(seq ${1:-3}); do for v in $2; do
  lib=""; [ "$v" != default ] && lib="--lib build/ab/$v.so"
  timeout -k 10 200 python bench.py $lib --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/abdrv_$v.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/abdrv_$v.log').read().strip().splitlines()[-1]);print('$v', round(d['value']), round(d['later_epochs']['value']))"
done; done

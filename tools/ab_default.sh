#!/bin/bash
# The driver's bench command (default launch sizes) alternating with a
# --split variant:  tools/ab_default.sh reps "10,10"
for r in $(seq ${1:-3}); do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/abd_default.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/abd_default.log').read().strip().splitlines()[-1]);print('default', round(d['value']), d['later_epochs']['value'], d['roofline']['launches'])"
  for v in $2; do
    timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --split $v > gpurun_out/abd_$v.log 2>&1 || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/abd_$v.log').read().strip().splitlines()[-1]);print('split $v', round(d['value']), d['later_epochs']['value'])"
  done
done

#!/bin/bash
# C5 at the driver's step count over launch groups: tools/ab_c5.sh reps "4 7 10"
for r in $(seq ${1:-2}); do for g in $2; do
  timeout -k 10 200 python bench.py --config c5 --steps 20 --warmup 5 --no-cpu-baseline --group $g > gpurun_out/c5g_$g.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/c5g_$g.log').read().strip().splitlines()[-1]);print('group $g', round(d['value']), d['config']['timed_launches'])"
done; done

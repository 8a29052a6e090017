#!/bin/bash
# Launch-size splits of the driver's 20 timed steps (bench --split), alternating:
#   tools/split_sweep.sh reps "10,10 12,8 ..." [bench args]
for r in $(seq ${1:-2}); do for v in $2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-later-epochs --split $v $3 > gpurun_out/split_${v}.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/split_${v}.log').read().strip().splitlines()[-1]);print('split $v', round(d['value']))"
done; done

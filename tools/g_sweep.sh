#!/bin/bash
# Launch-group sweep on one box: the driver's command (20 steps) and 400
# steps at several batches-per-launch, alternating.   tools/g_sweep.sh <tag>
set -e
TAG=${1:-gs}
mkdir -p gpurun_out
for rep in 1 2; do
  for g in 12 16 20 24; do
    for st in "20 5" "400 20"; do
      set -- $st
      timeout -k 10 200 python bench.py --steps $1 --warmup $2 --group $g --no-cpu-baseline --no-later-epochs > gpurun_out/${TAG}.tmp 2>&1
      python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}.tmp').read().strip().splitlines()[-1]); print('G', $g, 'steps', $1, 'rep', $rep, round(d['value']), d['config'].get('timed_launches'))" | tee -a gpurun_out/${TAG}.txt
    done
  done
done

#!/bin/bash
# Launch-group sweep, second pass: small groups for the 20-step command,
# larger for 400 steps.   tools/g_sweep2.sh <tag>
set -e
TAG=${1:-gs2}
mkdir -p gpurun_out
run() {
  timeout -k 10 200 python bench.py --steps $1 --warmup $2 --group $3 --inflight $4 --no-cpu-baseline --no-later-epochs > gpurun_out/${TAG}.tmp 2>&1
  python3 -c "import json,sys; d=json.loads(open('gpurun_out/${TAG}.tmp').read().strip().splitlines()[-1]); print('G', $3, 'inflight', $4, 'steps', $1, round(d['value']), d['config'].get('timed_launches'))" | tee -a gpurun_out/${TAG}.txt
}
for rep in 1 2; do
  for g in 4 5 7 10; do run 20 5 $g 3; done
  run 20 5 5 4; run 20 5 7 2
  for g in 20 32; do run 400 20 $g 3; done
  run 400 20 20 2
done

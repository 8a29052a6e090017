#!/bin/bash
# repeated driver-shaped runs on one box: the headline's spread (profiles/r8x_headline_spread.log)
set -e
for i in 1 2 3 4 5; do
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-later-epochs --no-c5 > gpurun_out/reps20_$i.log 2>&1
  python -c "import json;d=json.loads(open('gpurun_out/reps20_$i.log').read().strip().splitlines()[-1]);print('20', round(d['value']), d['parity']['mismatch'])"
done
for i in 1 2 3; do
  timeout -k 10 300 python bench.py --gpus 1 --no-cpu-baseline --no-later-epochs --no-c5 > gpurun_out/reps400_$i.log 2>&1
  python -c "import json;d=json.loads(open('gpurun_out/reps400_$i.log').read().strip().splitlines()[-1]);print('400', round(d['value']), d['parity']['mismatch'])"
done

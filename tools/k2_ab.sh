#!/bin/bash
# A/B the K2 staging variants (FFCV_K2_FLAGS) on the C3 bench, inflight 1 and 3.
for f in ${FLAGS:-0 1 2 3}; do
  for k in 1 3; do
    timeout -k 10 200 python bench.py --k2flags $f --dataset-size 65536 --steps 30 --warmup 5 --no-cpu-baseline --inflight $k > gpurun_out/ab_${f}_$k.log 2>&1 || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/ab_${f}_$k.log').read().strip().splitlines()[-1]);print('flags', $f, 'inflight', $k, d['value'])"
  done
done

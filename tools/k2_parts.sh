#!/bin/bash
# K2-only throughput with parts of the linear fast path skipped (timing only).
for f in 0 256 512 1024 1792; do
  timeout -k 10 200 python bench.py --k2flags $f --dataset-size 262144 --steps 100 --warmup 10 --no-cpu-baseline --only 4 > gpurun_out/k2p_$f.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/k2p_$f.log').read().strip().splitlines()[-1]);print('k2flags $f K2-only', d['value'])"
done

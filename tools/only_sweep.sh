#!/bin/bash
# Throughput with only a subset of the decode kernels in the timed steps
# (bench.py --only; timing only).   tools/only_sweep.sh "1 2 4 7" [inflight]
for m in ${1:-1 2 4 7}; do
  timeout -k 10 200 python bench.py --dataset-size 262144 --steps 100 --warmup 10 --no-cpu-baseline --inflight ${2:-8} --only $m > gpurun_out/only_$m.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/only_$m.log').read().strip().splitlines()[-1]);print('only', $m, 'inflight', ${2:-8}, d['value'], 'img/s', d['roofline']['kernel_ms'], 'ms/launch')"
done

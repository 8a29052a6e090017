#!/bin/bash
# C3 bench throughput vs GPU_MAX_HW_QUEUES x batches in flight.
#   tools/hwq_sweep.sh "16:6 16:8 24:12"
for qk in ${1:-4:3 8:4 16:8}; do
  q=${qk%%:*}; k=${qk##*:}
  GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --dataset-size 262144 --steps 60 --warmup 10 --no-cpu-baseline --inflight $k > gpurun_out/hwq_${q}_$k.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/hwq_${q}_$k.log').read().strip().splitlines()[-1]);print('hwq', $q, 'inflight', $k, d['value'])"
done

#!/bin/bash
# throughput vs (batch, inflight, HW queues), full decode and K1 only
#   tools/sweep_bq.sh "512:16:16 1024:8:8 ..."
for cfg in $1; do
  IFS=: read b k q <<< "$cfg"
  for only in 0 1; do
    GPU_MAX_HW_QUEUES=$q timeout -k 10 200 python bench.py --dataset-size 262144 --steps 80 --warmup 8 --no-cpu-baseline --batch $b --inflight $k --only $only > gpurun_out/sw_${b}_${k}_${q}_$only.log 2>&1 || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/sw_${b}_${k}_${q}_$only.log').read().strip().splitlines()[-1]);print('batch $b inflight $k hwq $q only $only', d['value'])"
  done
done

#!/bin/bash
# One GPU-box pass: parity tests, K1 phase stamps, bench at 1 and 3 batches in
# flight, optional SQ counters.  tools/gpu_check.sh <tag> [sq]
TAG=${1:-x}
mkdir -p gpurun_out
timeout -k 10 420 python -m pytest tests -q -m gpu -x > gpurun_out/t_$TAG.log 2>&1
rc=$?; tail -1 gpurun_out/t_$TAG.log
[ $rc -ne 0 ] && { tail -30 gpurun_out/t_$TAG.log; exit 1; }
timeout -k 10 120 python tools/jpeg_phases.py 512 > gpurun_out/ph_$TAG.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/ph_$TAG.log
for k in 1 3 4; do
  timeout -k 10 200 python bench.py --dataset-size 65536 --steps 30 --warmup 5 --no-cpu-baseline --inflight $k > gpurun_out/b${k}_$TAG.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/b${k}_$TAG.log').read().strip().splitlines()[-1]);print('inflight', $k, d['value'], 'img/s', d['ms_per_step'], 'ms/step', d['roofline']['kernel_ms'], 'ms/launch')"
done
if [ "$2" = sq ]; then bash tools/sq_counters.sh $TAG > /dev/null 2>&1 && python tools/sq_summary.py gpurun_out/sq_$TAG | head -16; fi

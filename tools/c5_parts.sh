#!/bin/bash
# C5 (raw RRC 448) rates of timing-only builds: tools/c5_parts.sh "default c5nostage ..." [reps]
for r in $(seq ${2:-1}); do for v in $1; do
  lib=""; [ $v != default ] && lib="--lib build/ab/$v.so"
  timeout -k 10 200 python bench.py $lib --config c5 --unique 1024 --steps 200 --warmup 20 --no-cpu-baseline --parity-rows 0 --no-host-check > gpurun_out/c5p_$v.log 2>&1 || { tail -3 gpurun_out/c5p_$v.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/c5p_$v.log').read().strip().splitlines()[-1]);print('$v', round(d['value']), round(1e9/d['value'],1), 'ns/img', d['roofline']['frac'])"
done; done

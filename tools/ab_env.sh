#!/bin/bash
# Alternating A/B of one environment knob of the library (read when a decoder
# context is made, e.g. FFCV_K1_ORDER) on the C3 bench:
#   tools/ab_env.sh <tag> <VAR> "<values>" <reps> [bench args]
TAG=$1; VAR=$2; VALS=$3; R=$4; shift 4
ARGS="--no-cpu-baseline --no-later-epochs --no-c5 --parity-rows 512 $@"
mkdir -p gpurun_out
for r in $(seq $R); do
  for v in $VALS; do
    f=gpurun_out/${TAG}_${VAR}_${v}_$r.log
    env $VAR=$v timeout -k 10 240 python bench.py $ARGS > $f 2>&1 || { tail -5 $f; exit 1; }
    python -c "
import json
d = json.loads(open('$f').read().strip().splitlines()[-1])
pk = d['roofline'].get('per_kernel', {})
print('$VAR=$v', round(d['value']), d['ms_per_step'], 'mismatch', d['parity']['mismatch'],
      {k: v.get('ns_per_image_isolated') for k, v in pk.items()})"
  done
done

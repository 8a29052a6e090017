#!/bin/bash
# K2 kernel choice A/B on the C3 bench: the library's size rule (default:
# band-loop kernel for launches of >= 8,192 images) vs FFCV_K2_LOOP=0
# (per-band kernel always), at the driver's 20 steps and at 400.
#   tools/ab_k2l.sh <tag> <reps>
TAG=${1:-k2l}; R=${2:-2}
mkdir -p gpurun_out
for r in $(seq $R); do
  for v in rule 0; do
    for st in 20 400; do
      w=20; [ $st = 20 ] && w=5
      f=gpurun_out/${TAG}_${v}_${st}_$r.log
      if [ $v = rule ]; then env -u FFCV_K2_LOOP timeout -k 10 240 python bench.py --no-cpu-baseline --no-later-epochs --no-c5 --parity-rows 256 --steps $st --warmup $w > $f 2>&1 || { tail -3 $f; exit 1; }
      else FFCV_K2_LOOP=$v timeout -k 10 240 python bench.py --no-cpu-baseline --no-later-epochs --no-c5 --parity-rows 256 --steps $st --warmup $w > $f 2>&1 || { tail -3 $f; exit 1; }; fi
      python -c "import json;d=json.loads(open('$f').read().strip().splitlines()[-1]);print('$v', '$st', round(d['value']), d['parity']['mismatch'])"
    done
  done
done

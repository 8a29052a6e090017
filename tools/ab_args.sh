#!/bin/bash
# Alternating A/B of bench.py argument sets on the C3 bench (the driver's 20
# steps unless the set says otherwise):
#   tools/ab_args.sh <tag> <reps> "name=args" "name=args" ...
#   e.g. tools/ab_args.sh sch 3 "base=" "k1s=--k1-streams 1 --split 8,8,4"
TAG=$1; R=$2; shift 2
BASE="--no-cpu-baseline --no-later-epochs --no-c5 --parity-rows 512 --steps 20 --warmup 5"
mkdir -p gpurun_out
for r in $(seq $R); do
  for set in "$@"; do
    name=${set%%=*}; args=${set#*=}
    f=gpurun_out/${TAG}_${name}_$r.log
    timeout -k 10 240 python bench.py $BASE $args > $f 2>&1 || { tail -5 $f; exit 1; }
    python -c "
import json
d = json.loads(open('$f').read().strip().splitlines()[-1])
print('$name', round(d['value']), d['ms_per_step'], 'mismatch', d['parity']['mismatch'], d['config'].get('timed_launches'))"
  done
done

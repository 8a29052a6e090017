#!/bin/bash
# K2-only rates isolating its fixed per-workgroup cost (timing-only flags).
set -e
OUT=gpurun_out/${1:-k2fixed}; mkdir -p $OUT
run() { timeout -k 10 200 python3 bench.py --steps 120 --warmup 12 --no-cpu-baseline --no-host-check --only 4 "${@:2}" > $OUT/$1.log 2>&1
  python3 -c "import json;d=json.loads(open('$OUT/$1.log').read().strip().splitlines()[-1]);print('$1', d['value'])"; }
run k2
run k2_fixed --k2flags 1792
run k2_fixed_nolut --k2flags 3840
run k2_band32 --lib build/ab/band32.so
run k2_band32_fixed --lib build/ab/band32.so --k2flags 1792
run k2_band8 --lib build/ab/band8.so
run full_band32 --lib build/ab/band32.so --only 7
echo DONE

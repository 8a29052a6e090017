#!/bin/bash
# A/B of library variants: K2-only and full C3 rates.  tools/ab_k2.sh <tag> v1 v2 ...
set -e
OUT=gpurun_out/${1}; shift; mkdir -p $OUT
for v in "$@"; do
  lib=""; [ "$v" != "base" ] && lib="--lib build/ab/$v.so"
  for only in 4 7; do
    timeout -k 10 200 python3 bench.py --steps 240 --warmup 12 --no-cpu-baseline --no-host-check --only $only $lib > $OUT/${v}_$only.log 2>&1
    python3 -c "import json;d=json.loads(open('$OUT/${v}_$only.log').read().strip().splitlines()[-1]);print('$v only=$only', d['value'])"
  done
done
echo AB_DONE

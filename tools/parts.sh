#!/bin/bash
# Per-kernel and per-K2-part rates (timing only: the flags skip work).
#   tools/parts.sh <tag> [extra bench args]
set -e
TAG=${1:-parts}; shift || true
OUT=gpurun_out/$TAG
mkdir -p $OUT
run() {  # name, args
  timeout -k 10 200 python3 bench.py --steps 120 --warmup 12 --no-cpu-baseline --no-host-check "${@:2}" > $OUT/$1.log 2>&1
  python3 -c "import json;d=json.loads(open('$OUT/$1.log').read().strip().splitlines()[-1]);print('$1', d['value'])"
}
run full "$@"
run k1 --only 1 "$@"
run k2 --only 4 "$@"
run k2_nocolour --only 4 --k2flags 256 "$@"
run k2_nowalk --only 4 --k2flags 512 "$@"
run k2_nostage --only 4 --k2flags 1024 "$@"
echo PARTS_DONE

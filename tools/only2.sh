#!/bin/bash
# One kernel alone (bench --only <bit>) for variants:  tools/only2.sh <bit> "v1 v2 ..." [reps]
B=$1; V=$2; R=${3:-1}
for r in $(seq $R); do for v in $V; do
  d=.; lib=""
  [ $v = old ] && d=build/ab/old_tree
  [ $v != old ] && [ $v != new ] && lib="--lib build/ab/$v.so"
  (cd $d && timeout -k 10 120 python bench.py $lib --only $B --steps 96 --warmup 24 --uniform-launches --no-cpu-baseline --no-later-epochs --no-host-check) > gpurun_out/o${B}_$v.log 2>&1 || { tail -3 gpurun_out/o${B}_$v.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/o${B}_$v.log').read().strip().splitlines()[-1]);print('$v only=$B', round(1e9/d['value'],1), 'ns/img')"
done; done

#!/bin/bash
# Kernel-alone rates (bench --only: the timed launches run only that kernel,
# on the scratch of earlier full launches) for trees/variants:
#   tools/only_ab.sh "old new w4"
for v in ${1:-old new}; do
  d=.; lib=""
  [ $v = old ] && d=build/ab/old_tree
  [ $v != old ] && [ $v != new ] && lib="--lib build/ab/$v.so"
  for o in 1 2 4; do
    (cd $d && timeout -k 10 120 python bench.py $lib --only $o --steps 96 --warmup 24 --uniform-launches --no-cpu-baseline --no-later-epochs --no-host-check) > gpurun_out/only_${v}_$o.log 2>&1 || { tail -3 gpurun_out/only_${v}_$o.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/only_${v}_$o.log').read().strip().splitlines()[-1]);print('$v only=$o', round(d['value']), 'img/s', round(1e9/d['value'],1), 'ns/img')"
  done
done

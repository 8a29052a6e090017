#!/bin/bash
# Alternating C3 A/B: `old` = a prebuilt old tree (build/ab/old_tree, e.g.
# `git archive <rev>` + its own build), `new` = the working tree, any other
# name = the working tree with --lib build/ab/<name>.so:
#   tools/ab_tree.sh "old new w4" <reps> [bench args]
V=${1:-"old new"}; R=${2:-2}; shift 2
ARGS="--no-cpu-baseline --no-later-epochs --parity-rows 256 $@"
for r in $(seq $R); do
  for v in $V; do
    d=.; lib=""
    [ $v = old ] && d=build/ab/old_tree
    [ $v != old ] && [ $v != new ] && lib="--lib build/ab/$v.so"
    (cd $d && timeout -k 10 240 python bench.py $lib $ARGS) > gpurun_out/abt_${v}_$r.log 2>&1 || { tail -5 gpurun_out/abt_${v}_$r.log; exit 1; }
    python -c "import json;d=json.loads(open('gpurun_out/abt_${v}_$r.log').read().strip().splitlines()[-1]);print('$v', round(d['value']), d['ms_per_step'], d.get('parity',{}).get('mismatch'))"
  done
done

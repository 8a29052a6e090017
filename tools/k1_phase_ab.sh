#!/bin/bash
# K1-alone rates (bench --only 1) of phase-stop builds in two trees:
#   tools/k1_phase_ab.sh "old:default old:old_s2 new:new_s4 new:eidx ..."
# tree old = build/ab/old_tree, new = .; variant default / eidx (entropy index:
# no sync pass) / <name> = --lib build/ab/<name>.so inside that tree
for spec in $1; do
  tree=${spec%%:*}; v=${spec#*:}; d=.; [ $tree = old ] && d=build/ab/old_tree
  lib=""; extra=""
  case $v in default) ;; eidx) extra="--entropy-index";; *) lib="--lib build/ab/$v.so";; esac
  (cd $d && timeout -k 10 200 python bench.py $lib $extra --no-cpu-baseline --no-later-epochs --only 1 --no-host-check --steps 200) > gpurun_out/k1pab_${tree}_$v.log 2>&1 || { tail -3 gpurun_out/k1pab_${tree}_$v.log; exit 1; }
  python -c "import json;d=json.loads(open('gpurun_out/k1pab_${tree}_$v.log').read().strip().splitlines()[-1]);print('$tree $v', round(d['value']), round(1e9/d['value'],1), 'ns/img')"
done

#!/bin/bash
# Alternating A/B of library builds on one box (C3 unless bench args say
# otherwise): each name is build/ab/<name>.so, or `new` = the working tree.
# Prints images/s, ms/step, parity mismatches and the three kernels'
# isolated ns per image from the line's per_kernel record.
#   tools/ab_libs.sh "base new" <reps> [bench args]
V=${1:-"base new"}; R=${2:-2}; shift 2
ARGS="--no-cpu-baseline --no-later-epochs --no-c5 --parity-rows 256 $@"
mkdir -p gpurun_out
for r in $(seq $R); do
  for v in $V; do
    lib=""; [ $v != new ] && lib="--lib build/ab/$v.so"
    f=gpurun_out/abl_${v}_$r.log
    timeout -k 10 300 python bench.py $lib $ARGS > $f 2>&1 || { tail -5 $f; exit 1; }
    python3 - $f $v <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
pk = d['roofline'].get('per_kernel', {})
ns = ' '.join(f"{k.split('<')[0].split('_')[1]}={v['ns_per_image_isolated']}" for k, v in pk.items())
print(sys.argv[2], round(d['value']), d['ms_per_step'], 'mismatch', d.get('parity', {}).get('mismatch'), ns, flush=True)
PY
  done
done

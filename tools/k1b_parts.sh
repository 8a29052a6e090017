#!/bin/bash
# jpeg_idct_kernel alone (bench --only 2) for timing-only builds without its DC
# phase / IDCT (build them with tools/build_variant.sh nodc -DK1B_SKIP_DC etc.
# on a tree whose K1b honours those macros):  tools/k1b_parts.sh reps
for r in $(seq ${1:-2}); do for v in default nodc noidct none; do
  lib=""; [ "$v" != default ] && lib="--lib build/ab/$v.so"
  timeout -k 10 200 python bench.py $lib --no-cpu-baseline --no-later-epochs --only 2 --no-host-check > gpurun_out/k1bp_$v.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/k1bp_$v.log').read().strip().splitlines()[-1]);print('$v', round(d['value']), round(1e9/d['value'],1), 'ns/img')"
done; done

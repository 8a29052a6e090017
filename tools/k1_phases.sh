#!/bin/bash
# K1-alone rates of timing-only builds that stop after a phase (K1_STOP,
# tools/build_variant.sh stopN -DK1_STOP=N), alternating:  tools/k1_phases.sh reps
for r in $(seq ${1:-2}); do
  for v in stop2 stop5 stop6 stop7 default eidx; do
    lib=""; extra=""
    case $v in default) ;; eidx) extra="--entropy-index";; *) lib="--lib build/ab/$v.so";; esac
    timeout -k 10 200 python bench.py $lib $extra --no-cpu-baseline --no-later-epochs --only 1 --no-host-check > gpurun_out/k1p_$v.log 2>&1 || exit 1
    python -c "import json;d=json.loads(open('gpurun_out/k1p_$v.log').read().strip().splitlines()[-1]);print('$v', round(d['value']), round(1e9/d['value'],1), 'ns/img')"
  done
done

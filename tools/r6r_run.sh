#!/bin/bash
# Round 6r: C5 row records from rrc_taps_kernel -- raw parity tests, C5 A/B against HEAD (build/ab/base.so)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py tests/test_loader_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "raw" > gpurun_out/r6r_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r6r_tests.log; [ $rc = 0 ] || exit 1
for r in 1 2 3; do for v in base new; do
  lib=""; [ $v != new ] && lib="--lib build/ab/$v.so"
  for sc in "--config c5" "--config c5 --draw-scale 0.08,0.4 --parity-rows 0"; do
    f=gpurun_out/r6r_${v}_${r}.log
    timeout -k 10 300 python bench.py $lib --no-cpu-baseline --no-later-epochs $sc > $f 2>&1 || { tail -5 $f; exit 1; }
    python3 - $f "$v $sc" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
r = d['roofline']
print(sys.argv[2], round(d['value']), 'kernel ns/img', r.get('kernel_ns_per_image_isolated'), 'frac', r.get('frac'), 'mismatch', d.get('parity', {}).get('mismatch'), flush=True)
PY
  done
done; done 2>&1 | tee gpurun_out/r6r_ab.log

#!/bin/bash
# Round 6i: C5 area column records from rrc_taps_kernel -- raw parity tests, C5 A/B against HEAD (build/ab/base.so)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "raw" > gpurun_out/r6i_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r6i_tests.log; [ $rc = 0 ] || exit 1
for r in 1 2; do for v in base new; do
  lib=""; [ $v != new ] && lib="--lib build/ab/$v.so"
  for sc in "" "--draw-scale 0.78,1.0 --parity-rows 0"; do
    f=gpurun_out/r6i_${v}_${r}.log
    timeout -k 10 300 python bench.py $lib --config c5 --no-cpu-baseline --no-later-epochs $sc > $f 2>&1 || { tail -5 $f; exit 1; }
    python3 - $f "$v $sc" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
r = d['roofline']
print(sys.argv[2], round(d['value']), 'kernel ns/img', r.get('kernel_ns_per_image_isolated'), 'frac', r.get('frac'), 'mismatch', d.get('parity', {}).get('mismatch'), flush=True)
PY
  done
done; done 2>&1 | tee gpurun_out/r6i_ab.log

#!/bin/bash
# Round 6j: area walks round by the 1.5 * 2^23 add -- parity (raw + JPEG RRC tests), C5 and C3 A/B against HEAD (build/ab/base.so)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "raw or rrc" > gpurun_out/r6j_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r6j_tests.log; [ $rc = 0 ] || exit 1
for r in 1 2; do for v in base new; do
  lib=""; [ $v != new ] && lib="--lib build/ab/$v.so"
  for sc in "--config c5" "--config c5 --draw-scale 0.78,1.0 --parity-rows 0" "--steps 100 --warmup 20 --no-c5 --draw-scale 0.85,1.0 --parity-rows 0"; do
    f=gpurun_out/r6j_${v}_${r}.log
    timeout -k 10 300 python bench.py $lib --no-cpu-baseline --no-later-epochs $sc > $f 2>&1 || { tail -5 $f; exit 1; }
    python3 - $f "$v $sc" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
r = d['roofline']
pk = r.get('per_kernel', {})
ns = ' '.join(f"{k.split('<')[0].split('_')[1]}={v['ns_per_image_isolated']}" for k, v in pk.items())
print(sys.argv[2], round(d['value']), 'kernel ns/img', r.get('kernel_ns_per_image_isolated'), ns, 'frac', r.get('frac'), 'mismatch', d.get('parity', {}).get('mismatch'), flush=True)
PY
  done
done; done 2>&1 | tee gpurun_out/r6j_ab.log

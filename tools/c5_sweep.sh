#!/bin/bash
# C5 raw-kernel build-parameter sweep: parity of each variant on the raw RRC
# tests, then a 400-step C5 bench per variant.  VARIANTS="default b8 ..."
# (variants built by tools/build_variant.sh into build/ab/).
set -e
mkdir -p gpurun_out
for v in ${VARIANTS:-default}; do
  lib=""; libarg=""; [ "$v" != default ] && lib=$PWD/build/ab/$v.so && libarg="--lib $lib"
  FFCV_HIP_LIB=$lib timeout -k 10 200 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
    tests/test_kernels_gpu.py -k raw_rrc > gpurun_out/c5sw_t_$v.log 2>&1
  echo "$v tests: $(tail -1 gpurun_out/c5sw_t_$v.log)"
  timeout -k 10 200 python bench.py $libarg --config c5 --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/c5sw_$v.log 2>&1
  python -c "import json;d=json.loads(open('gpurun_out/c5sw_$v.log').read().strip().splitlines()[-1]);print('$v', d['value'], 'img/s', d['roofline']['launch_ms'], 'ms/launch', d['roofline']['frac'])"
done

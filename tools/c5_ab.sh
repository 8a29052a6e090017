set -e
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_kernels_gpu.py -k "raw_rrc" > gpurun_out/c5_tests.log 2>&1
for v in ${VARIANTS:-default prev skiparea}; do
  lib=""; [ "$v" != default ] && lib=build/ab/$v.so
  timeout -k 10 200 python bench.py --lib $lib --config c5 --steps 400 --warmup 20 --no-cpu-baseline > gpurun_out/c5ab_$v.log 2>&1
  python -c "import json;d=json.loads(open('gpurun_out/c5ab_$v.log').read().strip().splitlines()[-1]);print('$v', d['value'], 'img/s', d['roofline']['kernel_ms'], 'ms/launch', d['roofline']['achieved'])"
done

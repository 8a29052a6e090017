set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r6d_tests.log 2>&1; tail -2 gpurun_out/r6d_tests.log
grep -q " passed" gpurun_out/r6d_tests.log && ! grep -q "FAILED" gpurun_out/r6d_tests.log || exit 1
bash tools/ab_libs.sh "base parse new" 2 --steps 20 --warmup 5 2>&1 | tee gpurun_out/r6d_ab20.log
bash tools/ab_libs.sh "base parse new" 1 2>&1 | tee gpurun_out/r6d_ab400.log
bash tools/c5_by_scale.sh r6d_c5s 2>&1 | tee gpurun_out/r6d_c5_by_scale.log

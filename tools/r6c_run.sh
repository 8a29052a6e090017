set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_photo.py -x -v --timeout 200 --timeout-method thread > gpurun_out/r6c_photo.log 2>&1; tail -2 gpurun_out/r6c_photo.log
bash tools/ab_libs.sh "base new" 3 --steps 20 --warmup 5 2>&1 | tee gpurun_out/r6c_ab20.log
bash tools/ab_libs.sh "base new" 2 2>&1 | tee gpurun_out/r6c_ab400.log

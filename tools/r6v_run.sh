#!/bin/bash
# Round 6v: K2 linear walk role-swapping sets -- GPU parity of the K2 paths, A/B against HEAD (build/ab/base.so)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_kernels_gpu.py tests/test_photo.py -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r6v_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r6v_tests.log; [ $rc = 0 ] || exit 1
bash tools/ab_libs.sh "base new" 2 --steps 20 --warmup 5 2>&1 | tee gpurun_out/r6v_ab20.log
bash tools/ab_libs.sh "base new" 2 2>&1 | tee gpurun_out/r6v_ab400.log

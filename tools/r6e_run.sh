#!/bin/bash
# Round 6e: K2 area walk -- GPU parity (area test first, then the suite), A/B against HEAD~ (build/ab/base.so)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 200 --timeout-method thread -k "rrc" > gpurun_out/r6e_rrc.log 2>&1; rc=$?; tail -3 gpurun_out/r6e_rrc.log; [ $rc = 0 ] || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r6e_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r6e_tests.log; [ $rc = 0 ] || exit 1
bash tools/ab_libs.sh "base new" 2 --steps 20 --warmup 5 2>&1 | tee gpurun_out/r6e_ab20.log
bash tools/ab_libs.sh "base new" 1 2>&1 | tee gpurun_out/r6e_ab400.log
bash tools/ab_libs.sh "base new" 1 --steps 100 --warmup 20 --draw-scale 0.85,1.0 --parity-rows 0 2>&1 | tee gpurun_out/r6e_ab_area.log

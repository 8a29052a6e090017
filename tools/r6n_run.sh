#!/bin/bash
# Round 6n: pooled later sync rounds (K1_POOL) -- K1 parity first (bounded), the GPU suite, then A/B against HEAD (build/ab/base.so)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 240 python -u -m pytest tests/test_kernels_gpu.py -m gpu -x -v --timeout 100 --timeout-method thread > gpurun_out/r6n_k.log 2>&1; rc=$?; tail -3 gpurun_out/r6n_k.log; [ $rc = 0 ] || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/r6n_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r6n_tests.log; [ $rc = 0 ] || exit 1
bash tools/ab_libs.sh "base new" 2 --steps 20 --warmup 5 2>&1 | tee gpurun_out/r6n_ab20.log
bash tools/ab_libs.sh "base new" 2 2>&1 | tee gpurun_out/r6n_ab400.log

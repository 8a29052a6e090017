#!/bin/bash
# Round-end evidence on one GPU box: gpu tests, C3/C5/C2 bench lines, rocprofv3
# kernel stats + FETCH/WRITE passes for C3 and C5.  tools/round_evidence.sh <tag>
set -e
TAG=${1:-r1i}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1
timeout -k 10 300 python bench.py --config c5 > gpurun_out/${TAG}_bench_c5.log 2>&1
timeout -k 10 300 python bench.py --config c2 --no-cpu-baseline > gpurun_out/${TAG}_bench_c2.log 2>&1
for f in bench bench_c5 bench_c2; do tail -1 gpurun_out/${TAG}_$f.log | cut -c1-160; done
bash tools/profile.sh ${TAG}_c3
bash tools/profile.sh ${TAG}_c5 --config c5 --steps 30 --warmup 5 --no-cpu-baseline

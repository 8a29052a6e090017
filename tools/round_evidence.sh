#!/bin/bash
# Round evidence on one GPU box: gpu tests, the driver's bench command, C3 /
# C5 / C2 400-step lines, the Loader rates, rocprofv3 kernel stats + FETCH /
# WRITE / SQ passes for C3 and C5.   tools/round_evidence.sh <tag>
set -e
TAG=${1:-r2a}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_driver.log 2>&1
timeout -k 10 300 python bench.py > gpurun_out/${TAG}_bench.log 2>&1
timeout -k 10 300 python bench.py --config c5 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_c5.log 2>&1
timeout -k 10 300 python bench.py --config c2 --steps 20 --warmup 5 --no-cpu-baseline > gpurun_out/${TAG}_bench_c2.log 2>&1
timeout -k 10 300 python bench.py --entropy-index --no-cpu-baseline > gpurun_out/${TAG}_bench_eidx.log 2>&1
for f in bench_driver bench bench_c5 bench_c2 bench_eidx; do tail -1 gpurun_out/${TAG}_$f.log | cut -c1-200; done
bash tools/profile.sh ${TAG}_c3 --steps 48 --warmup 12 --no-cpu-baseline
python3 tools/pmc_summary.py gpurun_out/prof_${TAG}_c3 6144 gpurun_out/${TAG}_c3_summary.json > /dev/null
bash tools/profile.sh ${TAG}_c5 --config c5 --steps 48 --warmup 12 --no-cpu-baseline
python3 tools/pmc_summary.py gpurun_out/prof_${TAG}_c5 1024 gpurun_out/${TAG}_c5_summary.json > /dev/null
if [ -n "$LOADER" ]; then
  timeout -k 10 600 python tools/loader_bench.py --n ${LOADER} > gpurun_out/${TAG}_loader.jsonl 2>&1
  cat gpurun_out/${TAG}_loader.jsonl
fi
echo EVIDENCE_DONE

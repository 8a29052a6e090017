#!/bin/bash
# Round evidence on one GPU box: gpu tests, the driver's bench command, C3 /
# C5 / C2 400-step lines, the Loader rates, rocprofv3 kernel stats + FETCH /
# WRITE / SQ passes for C3, C2 and C5, and a kernel trace of the driver's
# command.   tools/round_evidence.sh <tag> [all|bench|prof]  (bench / prof: the
# two halves, for two gpurun calls)
set -e
TAG=${1:-r4a}; PART=${2:-all}
mkdir -p gpurun_out
if [ $PART != prof ]; then
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > gpurun_out/${TAG}_tests.log 2>&1
tail -1 gpurun_out/${TAG}_tests.log
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/${TAG}_bench_driver.log 2>&1
timeout -k 10 300 python bench.py --no-c5 > gpurun_out/${TAG}_bench.log 2>&1
timeout -k 10 300 python bench.py --config c5 --steps 200 --warmup 20 --unique 1024 > gpurun_out/${TAG}_bench_c5.log 2>&1
timeout -k 10 300 python bench.py --config c2 --steps 200 --warmup 20 --unique 10000 > gpurun_out/${TAG}_bench_c2.log 2>&1
timeout -k 10 300 python bench.py --entropy-index --no-cpu-baseline --no-c5 > gpurun_out/${TAG}_bench_eidx.log 2>&1
# N > 1 rehearsal on one GPU: two ranks, gloo barrier (the driver's 8-GPU run uses RCCL)
FFCV_BENCH_BACKEND=gloo timeout -k 10 300 python bench.py --gpus 2 --steps 40 --warmup 10 --no-cpu-baseline --no-later-epochs > gpurun_out/${TAG}_bench_2rank.log 2>&1
for f in bench_driver bench bench_c5 bench_c2 bench_eidx bench_2rank; do tail -1 gpurun_out/${TAG}_$f.log | cut -c1-200; done
fi
[ $PART = bench ] && { echo EVIDENCE_DONE; exit 0; }
# every profiled launch the same size (C3 / C2: 24 batches per launch, warmup = one launch)
bash tools/profile.sh ${TAG}_c3 --steps 48 --warmup 24 --no-cpu-baseline --uniform-launches
python3 tools/pmc_summary.py gpurun_out/prof_${TAG}_c3 12288 gpurun_out/${TAG}_c3_summary.json gpurun_out/traffic_c3.json gpurun_out/sq_c3.json > /dev/null
bash tools/profile.sh ${TAG}_c2 --config c2 --unique 10000 --steps 48 --warmup 24 --no-cpu-baseline --uniform-launches
python3 tools/pmc_summary.py gpurun_out/prof_${TAG}_c2 6144 gpurun_out/${TAG}_c2_summary.json gpurun_out/traffic_c2.json gpurun_out/sq_c2.json > /dev/null
# C5 launches one at a time (--inflight 1): the profile's avg_ns is then the
# kernel's own duration, so the line's HBM fraction follows from it
bash tools/profile.sh ${TAG}_c5 --config c5 --unique 1024 --steps 40 --warmup 10 --no-cpu-baseline --uniform-launches --inflight 1
python3 tools/pmc_summary.py gpurun_out/prof_${TAG}_c5 2560 gpurun_out/${TAG}_c5_summary.json gpurun_out/traffic_c5.json gpurun_out/sq_c5.json > /dev/null
# kernel trace of the driver's command (tools/timeline.py)
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/trace_${TAG}_driver -o run -- python3 bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-later-epochs --no-c5 --no-host-check > gpurun_out/${TAG}_driver_traced.log 2>&1
if [ -n "$LOADER" ]; then
  timeout -k 10 600 python tools/loader_bench.py --n ${LOADER} > gpurun_out/${TAG}_loader.jsonl 2>&1
  cat gpurun_out/${TAG}_loader.jsonl
fi
echo EVIDENCE_DONE

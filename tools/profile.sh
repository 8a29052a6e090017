#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box from the repo root).
#   tools/profile.sh <tag> [bench args...]
# Pass 1: --kernel-trace --stats (per-kernel durations).
# Pass 2/3: PMC FETCH_SIZE and WRITE_SIZE in separate passes (never combined
# with tracing domains; MI355X_MICROARCH.md rocprofv3 section).
set -e
TAG=${1:-r1}; shift || true
ARGS=${@:---dataset-size 262144 --steps 30 --warmup 5 --no-cpu-baseline}
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
# the profiler's preload initialises HIP before bench.py can raise the queue count
export GPU_MAX_HW_QUEUES=16
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1
echo PROFILE_DONE

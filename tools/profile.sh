#!/bin/bash
# rocprofv3 evidence for bench.py (run on the GPU box from the repo root).
#   tools/profile.sh <tag> [bench args...]
# Pass 1: --kernel-trace --stats (per-kernel durations).
# Pass 2/3: PMC FETCH_SIZE and WRITE_SIZE in separate passes (never combined
# with tracing domains; MI355X_MICROARCH.md rocprofv3 section).
# Pass 4: SQ instruction / wait counters (8 SQ slots, one pass).
# Use --steps / --warmup that are multiples of the config's batches per
# launch and --uniform-launches so every launch has the same size
# (tools/pmc_summary.py divides by it).
set -e
TAG=${1:-r2}; shift || true
ARGS="${@:---steps 48 --warmup 12 --no-cpu-baseline} --no-host-check --no-later-epochs"
OUT=gpurun_out/prof_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/trace -o run -- python3 bench.py $ARGS > $OUT/trace.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $OUT/fetch -o run -- python3 bench.py $ARGS > $OUT/fetch.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d $OUT/write -o run -- python3 bench.py $ARGS > $OUT/write.log 2>&1
timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM --output-format csv -d $OUT/sq -o run -- python3 bench.py $ARGS > $OUT/sq.log 2>&1
echo PROFILE_DONE

#!/bin/bash
# SQ instruction/stall counters for the bench kernels (GPU box, repo root).
#   tools/sq_counters.sh <tag> [bench args...]
# Two PMC passes (8 SQ slots each), no tracing domains combined with --pmc.
set -e
TAG=${1:-sq}; shift || true
ARGS=${@:---dataset-size 65536 --steps 10 --warmup 3 --no-cpu-baseline}
OUT=gpurun_out/sq_$TAG
mkdir -p $OUT
export TMPDIR=/tmp
export GPU_MAX_HW_QUEUES=16
timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU --output-format csv -d $OUT/p1 -o run -- python3 bench.py $ARGS > $OUT/p1.log 2>&1
timeout -k 10 300 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INST_CYCLES_VMEM --output-format csv -d $OUT/p2 -o run -- python3 bench.py $ARGS > $OUT/p2.log 2>&1
echo SQ_DONE

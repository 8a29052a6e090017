#!/bin/bash
# Instruction-fetch counters per kernel (one --pmc pass).
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16
OUT=gpurun_out/icache; rm -rf $OUT; mkdir -p $OUT
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_IFETCH SQ_WAIT_INST_ANY SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d $OUT -o run -- python3 bench.py --dataset-size 65536 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/log 2>&1
rc=$?; tail -3 $OUT/log; [ $rc = 0 ] || exit $rc
python3 tools/sq_report.py $OUT icache

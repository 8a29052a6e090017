#!/bin/bash
# Instruction-fetch counters per kernel (per wave): K1 alone (--only 1) and the
# full C3 pipeline.  Two passes each: SQ_ wave/fetch counters, then SQC_ I-cache.
export TMPDIR=/tmp
for mode in only1 full; do
  extra=""; [ $mode = only1 ] && extra="--only 1"
  for pass in sq sqc; do
    if [ $pass = sq ]; then P="SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_IFETCH SQ_WAIT_ANY SQ_ACTIVE_INST_ANY"; else P="SQ_WAVES SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQC_ICACHE_MISSES_DUPLICATE"; fi
    OUT=gpurun_out/ic_${mode}_$pass; rm -rf $OUT; mkdir -p $OUT
    timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d $OUT -o run -- python3 bench.py $extra --steps 48 --warmup 24 --uniform-launches --no-cpu-baseline --no-host-check --no-later-epochs --parity-rows 0 > $OUT/log 2>&1 || exit 1
    python3 tools/sq_report.py $OUT ${mode}_$pass jpeg || exit 1
  done
done

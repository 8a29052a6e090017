#!/bin/bash
# SQ instruction counters (one --pmc pass) per library variant, K1/K2 per wave.
#   tools/sq_ab.sh "base default ..."   (variants as in tools/ab.sh)
export TMPDIR=/tmp GPU_MAX_HW_QUEUES=16
for v in $1; do
  lib=""; [ "$v" != default ] && lib=$PWD/build/ab/$v.so
  OUT=gpurun_out/sqab_$v; rm -rf $OUT; mkdir -p $OUT
  FFCV_HIP_LIB=$lib timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_BRANCH --output-format csv -d $OUT -o run -- python3 bench.py --dataset-size 65536 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/log 2>&1 || exit 1
  python3 tools/sq_report.py $OUT $v || exit 1
done

#!/bin/bash
# SQ counters per wave of the raw C5 kernel for library variants (one --pmc pass each):
#   tools/c5_sq.sh "default head ..."
export TMPDIR=/tmp
for v in $1; do
  lib=""; [ "$v" != default ] && lib="--lib build/ab/$v.so"
  OUT=gpurun_out/c5sq_$v; rm -rf $OUT; mkdir -p $OUT
  timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM --output-format csv -d $OUT -o run -- python3 bench.py $lib --config c5 --unique 1024 --steps 40 --warmup 10 --group 4 --uniform-launches --no-cpu-baseline --parity-rows 0 --no-host-check --no-later-epochs > $OUT/log 2>&1 || exit 1
  python3 tools/sq_report.py $OUT $v rrc_raw || exit 1
done

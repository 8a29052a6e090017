#!/bin/bash
# K2-only SQ counters per wave for the timing-only part flags (0 full, 256 no
# colour pass, 512 no column walk, 1024 no tile staging loads, 1792 none):
#   tools/k2_sq.sh "0 256 512 1024 1792"
export TMPDIR=/tmp
for f in ${1:-0 256 512 1024 1792}; do
  OUT=gpurun_out/k2sq_$f; rm -rf $OUT; mkdir -p $OUT
  timeout -s KILL 300 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VMEM --output-format csv -d $OUT -o run -- python3 bench.py ${LIB:+--lib $LIB} --k2flags $f --dataset-size 65536 --unique 16384 --steps 48 --warmup 24 --uniform-launches --no-cpu-baseline --only 4 --no-host-check --no-later-epochs --parity-rows 0 > $OUT/log 2>&1 || exit 1
  python3 tools/sq_report.py $OUT k2flags=$f color_resize || exit 1
done

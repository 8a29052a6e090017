#!/bin/bash
# Issue / LDS / TA counters of the timed launches of one kernel alone
# (--only 1: K1, --only 4: K2), two --pmc passes each: tools/sq_deep.sh <tag>
export TMPDIR=/tmp
OUT=gpurun_out/${1:-sqdeep}; mkdir -p $OUT
P1="SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_VMEM SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_BUSY_CYCLES"
P2="SQ_THREAD_CYCLES_VALU SQ_INST_CYCLES_VMEM_RD SQ_INST_CYCLES_VMEM_WR SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_ADDR_CONFLICT SQ_INSTS_VALU SQ_WAVE_CYCLES"
for o in 1 4; do
  for p in 1 2; do
    eval C=\$P$p
    timeout -s KILL 120 rocprofv3 --pmc $C --output-format csv -d $OUT/o${o}p$p -o run -- python3 bench.py --steps 48 --warmup 12 --no-cpu-baseline --no-host-check --no-later-epochs --only $o > $OUT/o${o}p$p.log 2>&1 || exit 1
  done
done
python3 - $OUT <<'PY'
import collections, csv, sys
d = sys.argv[1]
for o, kname in (('1', 'jpeg_entropy_kernel'), ('4', 'jpeg_color_resize_kernel')):
    m = {}
    for p in ('1', '2'):
        rows = collections.defaultdict(dict)
        for r in csv.DictReader(open(f'{d}/o{o}p{p}/run_counter_collection.csv')):
            if kname in r['Kernel_Name']:
                rows[int(r['Dispatch_Id'])][r['Counter_Name']] = float(r['Counter_Value'])
        last = [rows[k] for k in sorted(rows)[-4:]]
        for n in last[0]:
            m[n] = sum(x[n] for x in last) / len(last) / 6144
    print(kname, 'per image:', {n: round(v) for n, v in sorted(m.items())})
PY

#!/bin/bash
# Instruction-fetch and issue-stall counters per kernel (one --pmc pass each).
#   tools/icache.sh <tag>
set -e
export TMPDIR=/tmp
TAG=${1:-icache}
OUT=gpurun_out/$TAG; rm -rf $OUT; mkdir -p $OUT
ARGS="--steps 48 --warmup 12 --no-cpu-baseline --no-host-check"
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_IFETCH SQ_WAIT_INST_ANY SQ_INSTS_SMEM SQC_ICACHE_HITS SQC_ICACHE_MISSES --output-format csv -d $OUT/p1 -o run -- python3 bench.py $ARGS > $OUT/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_ACTIVE_INST_ANY --output-format csv -d $OUT/p2 -o run -- python3 bench.py $ARGS > $OUT/p2.log 2>&1
python3 - $OUT <<'PY'
import collections, csv, sys
d = sys.argv[1]
agg = collections.defaultdict(lambda: collections.defaultdict(list))
for p in ('p1', 'p2'):
    for r in csv.DictReader(open(f'{d}/{p}/run_counter_collection.csv')):
        agg[r['Kernel_Name'].split('(')[0]][r['Counter_Name']].append(float(r['Counter_Value']))
for k, c in agg.items():
    if 'jpeg' not in k and 'rrc' not in k:
        continue
    m = {n: sum(v) / len(v) for n, v in c.items()}
    w = m.get('SQ_WAVES', 1)
    print(k, 'waves/launch', w)
    for n in sorted(m):
        print(f'   {n:22s} {m[n]:16.0f}  per-wave {m[n] / w:12.1f}')
PY
echo ICACHE_DONE

#!/bin/bash
# K1's cycles by instruction class and wait reason: three SQ passes (8 SQ
# counters each, one rocprofv3 run per pass) over K1-only launches of 12,288
# images (bench.py --only 1), printed per image.   tools/k1_stalls.sh <tag>
TAG=${1:-k1s}
mkdir -p gpurun_out
export TMPDIR=/tmp
# samples generated (and cached in /tmp) outside the profiler (see k1_phase_valu.sh)
timeout -k 10 600 python3 -c "import bench; bench.make_unique('jpg', 256, 65536, 0, 16)" || exit 1
P1="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_MISC"
P2="SQ_WAVES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_ADDR_CONFLICT SQ_INST_CYCLES_SALU SQ_THREAD_CYCLES_VALU"
P3="SQ_WAVES SQ_INSTS_SMEM SQ_INST_CYCLES_SMEM SQ_INSTS_BRANCH SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_IFETCH"
i=0
for P in "$P1" "$P2" "$P3"; do
  i=$((i + 1))
  timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d gpurun_out/${TAG}_p$i -o run -- python3 bench.py --only 1 --steps 48 --warmup 24 --no-cpu-baseline --uniform-launches --no-host-check --no-later-epochs --no-c5 --parity-rows 0 --no-kernel-events > gpurun_out/${TAG}_p$i.log 2>&1 || { tail -3 gpurun_out/${TAG}_p$i.log; exit 1; }
done
python3 - <<PY
import csv, collections
for i in (1, 2, 3):
    v = collections.defaultdict(lambda: collections.defaultdict(float))
    for r in csv.DictReader(open('gpurun_out/${TAG}_p%d/run_counter_collection.csv' % i)):
        if 'entropy' not in r['Kernel_Name']:
            continue
        v[r['Counter_Name']][r['Dispatch_Id']] += float(r['Counter_Value'])
    for c, d in sorted(v.items()):
        x = list(d.values())
        print(c, 'per image %.0f' % (sum(x) / len(x) / 12288), 'launches', len(x))
PY

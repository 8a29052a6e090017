#!/bin/bash
# Launch-shape sweep of bench.py on one GPU box (repo root):
#   tools/sweep_group.sh <tag> [groups] [inflights] [configs]
# 1) the driver's exact command, 2) batches-per-launch x launches-in-flight at
# the driver's step count and at 400 steps.  HIP's default hardware queues.
set -e
TAG=${1:-sw}
GS=${2:-"6 8 12"}
SS=${3:-"2 3 4"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/driver.log 2>&1
tail -1 $OUT/driver.log | cut -c1-300
for g in $GS; do
  for s in $SS; do
    for k in 20 400; do
      timeout -k 10 200 python3 bench.py --steps $k --warmup 5 --group $g --inflight $s --no-cpu-baseline > $OUT/g${g}_s${s}_k${k}.log 2>&1
      python3 -c "import json,sys;d=json.loads(open('$OUT/g${g}_s${s}_k${k}.log').read().strip().splitlines()[-1]);print('G=$g S=$s K=$k', d['value'], d['ms_per_step'], d['host_submit_ms_per_step'], d['roofline']['launch_ms'])"
    done
  done
done
for c in c5 c2; do
  timeout -k 10 300 python3 bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline > $OUT/$c.log 2>&1
  python3 -c "import json,sys;d=json.loads(open('$OUT/$c.log').read().strip().splitlines()[-1]);print('$c K=20', d['value'], d['ms_per_step'], d['roofline']['launch_ms'])"
done
echo SWEEP_DONE

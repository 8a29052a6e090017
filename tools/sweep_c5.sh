#!/bin/bash
# C5 launch-shape sweep (raw RRC 448 + Cutout 64, batch 256).
set -e
OUT=gpurun_out/${1:-c5sw}; mkdir -p $OUT
for g in 1 2 4 8; do for s in 2 3 4; do for k in 20 400; do
  timeout -k 10 200 python3 bench.py --config c5 --steps $k --warmup 5 --group $g --inflight $s --no-cpu-baseline --no-host-check > $OUT/g${g}_s${s}_k${k}.log 2>&1
  python3 -c "import json;d=json.loads(open('$OUT/g${g}_s${s}_k${k}.log').read().strip().splitlines()[-1]);print('G=$g S=$s K=$k', d['value'], d['host_submit_ms_per_step'], d['ms_per_step'])"
done; done; done
echo C5_DONE

#!/bin/bash
# Round 6s: final-build check -- GPU suite, smoke(), and five driver-shaped runs (spread)
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread > gpurun_out/r6s_tests.log 2>&1; rc=$?; tail -2 gpurun_out/r6s_tests.log; [ $rc = 0 ] || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('SMOKE_OK')" > gpurun_out/r6s_smoke.log 2>&1; rc=$?; tail -1 gpurun_out/r6s_smoke.log; [ $rc = 0 ] || exit 1
for r in 1 2 3 4 5; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline --no-later-epochs --no-c5 > gpurun_out/r6s_drv_$r.log 2>&1 || { tail -3 gpurun_out/r6s_drv_$r.log; exit 1; }
  python3 -c "import json;d=json.loads([l for l in open('gpurun_out/r6s_drv_$r.log') if l.startswith('{')][-1]);print('driver-shaped', round(d['value']), d['ms_per_step'], 'mismatch', d['parity']['mismatch'])"
done 2>&1 | tee gpurun_out/r6s_spread.log

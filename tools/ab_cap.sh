#!/bin/bash
# Driver command variants alternating on one box: tools/ab_cap.sh reps "name:args" ...
reps=$1; shift
for r in $(seq $reps); do for spec in "$@"; do
  name=${spec%%:*}; args=${spec#*:}
  timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 --no-cpu-baseline $args > gpurun_out/abc_$name.log 2>&1 || exit 1
  python -c "import json;d=json.loads(open('gpurun_out/abc_$name.log').read().strip().splitlines()[-1]);print('$name', round(d['value']), d['later_epochs']['value'])"
done; done

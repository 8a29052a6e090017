#!/bin/bash
# C5 (raw 512^2 -> 448) time per image by crop-scale band (VERDICT r5 next 5:
# split the linear walk's time by input class).  Each band: crops of area
# scale in [lo, hi] of the 512^2 image with ratio 1, launches one at a time
# (--inflight 1), the raw kernel's isolated ns per image from the line.
#   tools/c5_by_scale.sh <tag>
TAG=${1:-c5s}
mkdir -p gpurun_out
for b in 0.08,0.15 0.15,0.25 0.25,0.40 0.40,0.60 0.60,0.76 0.78,1.0; do
  f=gpurun_out/${TAG}_$b.log
  timeout -k 10 300 python bench.py --config c5 --unique 1024 --steps 40 --warmup 10 --no-cpu-baseline --no-later-epochs --parity-rows 0 --inflight 1 --draw-scale $b > $f 2>&1 || { tail -3 $f; exit 1; }
  python3 - $f $b <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
r = d['roofline']
print('scale', sys.argv[2], 'images/s', round(d['value']), 'kernel ns/img', r.get('kernel_ns_per_image_isolated'),
      'alg bytes/img', r.get('algorithmic_bytes_per_image'), 'hbm frac', r.get('frac'), flush=True)
PY
done

#!/bin/bash
# C3 rocprofv3 stats + FETCH / WRITE / SQ passes of the in-tree build, uniform
# 12,288-image launches:  tools/prof_c3.sh <tag>
TAG=${1:-r2k}
bash tools/profile.sh ${TAG}_c3 --steps 48 --warmup 24 --no-cpu-baseline --uniform-launches > gpurun_out/${TAG}_prof.log 2>&1 || exit 1
python3 tools/pmc_summary.py gpurun_out/prof_${TAG}_c3 12288 gpurun_out/${TAG}_c3_summary.json gpurun_out/traffic_c3.json gpurun_out/sq_c3.json > /dev/null || exit 1
python3 - "$TAG" <<'PY'
import json, sys
d = json.load(open(f'gpurun_out/{sys.argv[1]}_c3_summary.json'))
for k, v in d.items():
    if 'jpeg' in k:
        print(k, v.get('calls'), round(v.get('avg_ns', 0) / 1e3, 1), 'us', round(v.get('valu_per_image', 0)), 'valu/img',
              round(v.get('hbm_bytes_per_image', 0)), 'B/img', 'wait', round(v.get('SQ_WAIT_ANY', 0) / max(1, v.get('SQ_WAVE_CYCLES', 1)), 3))
PY

"""Summarise a tools/profile.sh run.

    python tools/pmc_summary.py gpurun_out/prof_<tag> <images_per_launch> \
        profiles/<tag>_summary.json [profiles/traffic_<cfg>.json profiles/sq_<cfg>.json]

Per kernel: launches, mean duration (kernel-trace pass), mean FETCH_SIZE /
WRITE_SIZE per launch from the two separate PMC passes (rocprofv3 reports
KB = 1024 B), the SQ counters per launch, and everything per image
(divided by the images per launch, which the profile run keeps constant).
Per MI355X_MICROARCH.md "HBM": gfx950 FETCH_SIZE counts 64 B per 128-B
request of wide (16 B/lane) streaming reads, so those read half their
bytes; the JPEG kernels read with byte/dword loads (no correction applied);
the raw kernel's 16-byte staging loads are the wide case (x2 noted).
The optional traffic_/sq_ files are what bench.py reads for its roofline.
"""
import collections
import csv
import json
import os
import sys

d, imgs, out = sys.argv[1], float(sys.argv[2]), sys.argv[3]
traffic_out = sys.argv[4] if len(sys.argv) > 4 else None
sq_out = sys.argv[5] if len(sys.argv) > 5 else None


def kname(n):
    return n.split('(')[0].replace('void ', '').strip()


res = collections.defaultdict(dict)
with open(os.path.join(d, 'trace', 'run_kernel_stats.csv')) as f:
    for r in csv.DictReader(f):
        res[kname(r['Name'])].update(calls=int(r['Calls']), avg_ns=float(r['AverageNs']))
for tag in ('fetch', 'write', 'sq'):
    path = os.path.join(d, tag, 'run_counter_collection.csv')
    if not os.path.exists(path):
        continue
    vals = collections.defaultdict(lambda: collections.defaultdict(list))
    with open(path) as f:
        for r in csv.DictReader(f):
            vals[kname(r['Kernel_Name'])][r['Counter_Name']].append(float(r['Counter_Value']))
    for k, cs in vals.items():
        for c, v in cs.items():
            res[k][c] = sum(v) / len(v)
def _ours(k):
    return k.startswith(('jpeg_', 'rrc_', 'lut_', 'draw_', 'gather_samples', 'gather_raw', 'cutout_', 'flip_'))


summary = {}
for k, v in res.items():
    e = dict(v)
    e['images'] = imgs
    if 'FETCH_SIZE' in e:
        e['fetch_size_kb'] = e.pop('FETCH_SIZE')
    if 'WRITE_SIZE' in e:
        e['write_size_kb'] = e.pop('WRITE_SIZE')
    if 'fetch_size_kb' in e and 'write_size_kb' in e:
        e['hbm_bytes_per_image'] = (e['fetch_size_kb'] + e['write_size_kb']) * 1024 / imgs
    if 'SQ_INSTS_VALU' in e:
        e['valu_per_image'] = e['SQ_INSTS_VALU'] / imgs
        e['salu_per_image'] = e.get('SQ_INSTS_SALU', 0) / imgs
    summary[k] = e
json.dump(summary, open(out, 'w'), indent=1, sort_keys=True)
print(json.dumps(summary, indent=1, sort_keys=True))
build = os.environ.get('FFCV_BUILD_TAG', os.path.basename(out).split('_')[0])
if traffic_out:
    json.dump({k: {x: v[x] for x in ('fetch_size_kb', 'write_size_kb', 'images', 'avg_ns') if x in v}
               for k, v in summary.items() if _ours(k)} | {'_build': build}, open(traffic_out, 'w'), indent=1,
              sort_keys=True)
if sq_out:
    json.dump({k: {x: v[x] for x in ('valu_per_image', 'salu_per_image', 'images', 'SQ_WAVES', 'SQ_INSTS_VALU',
                                     'SQ_WAVE_CYCLES', 'SQ_WAIT_ANY', 'SQ_ACTIVE_INST_ANY', 'avg_ns') if x in v}
               for k, v in summary.items() if 'valu_per_image' in v and _ours(k)} | {'_build': build},
              open(sq_out, 'w'), indent=1, sort_keys=True)

"""Summarise a tools/profile.sh run into profiles/<tag>_summary.json.

    python tools/pmc_summary.py gpurun_out/prof_<tag> profiles/<tag>_summary.json

Per kernel: launches, mean duration (kernel-trace pass), and mean FETCH_SIZE /
WRITE_SIZE per launch from the two separate PMC passes.  rocprofv3 reports
both in KB (1024 B).  Per MI355X_MICROARCH.md "HBM": gfx950 FETCH_SIZE counts
64 B per 128-B request of wide (16 B/lane) streaming reads, so those read
half their bytes; narrower access widths are uncalibrated.  The decode
kernels read with byte/dword loads, so no correction is applied and the
figures are reported as measured.
"""
import collections
import csv
import json
import os
import sys

d, out = sys.argv[1], sys.argv[2]


def kname(n):
    return n.split('(')[0].replace('void ', '').strip()


res = collections.defaultdict(dict)
with open(os.path.join(d, 'trace', 'run_kernel_stats.csv')) as f:
    for r in csv.DictReader(f):
        res[kname(r['Name'])].update(calls=int(r['Calls']), avg_ns=float(r['AverageNs']))
for tag, counter in (('fetch', 'FETCH_SIZE'), ('write', 'WRITE_SIZE')):
    vals = collections.defaultdict(list)
    with open(os.path.join(d, tag, 'run_counter_collection.csv')) as f:
        for r in csv.DictReader(f):
            if r['Counter_Name'] == counter:
                vals[kname(r['Kernel_Name'])].append(float(r['Counter_Value']))
    for k, v in vals.items():
        res[k][counter.lower() + '_kb'] = sum(v) / len(v)
json.dump(dict(res), open(out, 'w'), indent=1, sort_keys=True)
print(json.dumps(dict(res), indent=1, sort_keys=True))

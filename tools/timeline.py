"""Timeline of the last N decode kernels in a rocprofv3 kernel trace:
    python tools/timeline.py gpurun_out/tl_drv [n_kernels]
Prints each kernel's queue, start and end relative to the first one (us) and
how long the GPU ran one kernel only / none in that window."""
import csv
import glob
import sys

d = sys.argv[1]
n = int(sys.argv[2]) if len(sys.argv) > 2 else 9
path = glob.glob(f'{d}/**/*kernel_trace.csv', recursive=True)[0]
rows = [r for r in csv.DictReader(open(path)) if 'jpeg' in r['Kernel_Name']]
rows.sort(key=lambda r: int(r['Start_Timestamp']))
rows = rows[-n:]
t0 = int(rows[0]['Start_Timestamp'])
ev = []
for r in rows:
    s, e = int(r['Start_Timestamp']) - t0, int(r['End_Timestamp']) - t0
    name = r['Kernel_Name'].split('(')[0].replace('void ', '')
    print(f"{name:40s} q{r.get('Queue_Id', '?'):>3s} {s / 1e3:9.1f} {e / 1e3:9.1f} {(e - s) / 1e3:8.1f}")
    ev += [(s, 1), (e, -1)]
ev.sort()
active, last, alone, idle = 0, 0, 0, 0
for t, dlt in ev:
    if active == 1:
        alone += t - last
    if active == 0:
        idle += t - last
    active += dlt
    last = t
print(f'window {last / 1e3:.1f} us: one kernel only {alone / 1e3:.1f} us, none {idle / 1e3:.1f} us')

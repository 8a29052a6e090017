"""Kernel concurrency over the timed region of a rocprofv3 kernel trace:
time-weighted number of in-flight kernels per name, and busy fractions.
    python tools/trace_conc.py <run_kernel_trace.csv> [last_n_dispatches]"""
import csv, sys, collections
rows = list(csv.DictReader(open(sys.argv[1])))
ev = []
for r in rows:
    n = r['Kernel_Name'].split('(')[0].replace('void ', '')
    s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
    ev.append((s, e, n, r['Queue_Id']))
ev.sort()
# argv[2]: analyse only the last N dispatches (the timed region)
if len(sys.argv) > 2:
    ev = ev[-int(sys.argv[2]):]
names = sorted(set(x[2] for x in ev))
pts = []
for s, e, n, q in ev:
    pts.append((s, 1, n)); pts.append((e, -1, n))
pts.sort()
cur = collections.Counter(); acc = collections.Counter(); busy = collections.Counter()
last = pts[0][0]; tot = 0; hist = collections.Counter()
for t, d, n in pts:
    dt = t - last
    if dt > 0:
        for k, v in cur.items():
            acc[k] += v * dt
            if v: busy[k] += dt
        hist[sum(cur.values())] += dt
        tot += dt
    cur[n] += d; last = t
print(f'span {tot/1e6:.2f} ms, queues {len(set(x[3] for x in ev))}')
for k in names:
    print(f'  {k[:40]:40s} mean in flight {acc[k]/tot:5.2f}  busy {busy[k]/tot:5.2f}')
print('  total in-flight histogram (fraction of time):', {k: round(v / tot, 3) for k, v in sorted(hist.items())})

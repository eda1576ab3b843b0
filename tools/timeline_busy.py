"""Busy fraction / concurrency of a rocprofv3 kernel trace (run on a bench trace).
usage: python tools/timeline_busy.py <kernel_trace.csv> [skip_first_ms]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
skip = float(sys.argv[2]) if len(sys.argv) > 2 else 0.0
iv = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
t0 = iv[0][0] + skip * 1e6
iv = [x for x in iv if x[0] >= t0]
ev = []
for s, e, _ in iv:
    ev.append((s, 1))
    ev.append((e, -1))
ev.sort()
depth, last, busy, acc = 0, ev[0][0], 0, defaultdict(int)
for t, d in ev:
    if depth > 0:
        busy += t - last
    acc[depth] += t - last
    depth += d
    last = t
span = ev[-1][0] - ev[0][0]
tot = sum(e - s for s, e, _ in iv)
print(f"span {span/1e6:.2f} ms, busy {busy/span:.3f}, summed kernel time / span {tot/span:.3f}")
for d in sorted(acc):
    print(f"  depth {d}: {acc[d]/span:.3f}")
per = defaultdict(float)
for s, e, n in iv:
    per[n.split("(")[0][:90]] += (e - s) / 1e3
for n, v in sorted(per.items(), key=lambda x: -x[1])[:25]:
    print(f"  {v/1e3:8.2f} ms  {n}")

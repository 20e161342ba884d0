"""Idle-gap report of a rocprofv3 kernel trace: GPU idle time (union of queues) in a window,
attributed to the kernel that ends each gap.  python scripts/gap_report.py trace.csv [start-substring]"""
import csv
import sys
from collections import defaultdict

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:80]) for r in rows)
start = sys.argv[2] if len(sys.argv) > 2 else None
if start:
    i0 = next(i for i, k in enumerate(ks) if start in k[2])
    ks = ks[i0:]
t0, t1 = ks[0][0], max(k[1] for k in ks)
busy_end = t0
gaps = defaultdict(lambda: [0, 0.0])
idle = 0.0
big = []
prev = ""
for s, e, n in ks:
    if s > busy_end:
        gaps[n][0] += 1
        gaps[n][1] += (s - busy_end) / 1e3
        idle += (s - busy_end) / 1e3
        if s - busy_end > 1_000_000:
            big.append(((s - busy_end) / 1e6, prev, n))
    busy_end = max(busy_end, e)
    prev = n
print(f"window {(t1 - t0) / 1e6:.1f} ms, idle {idle / 1e3:.1f} ms ({100 * idle / ((t1 - t0) / 1e3):.0f} %)")
for n, (c, us) in sorted(gaps.items(), key=lambda x: -x[1][1])[:20]:
    print(f"{us / 1e3:9.2f} ms {c:6d}  before {n}")
print("gaps > 1 ms (after -> before):")
for ms, a, b in big[:12]:
    print(f"  {ms:7.2f} ms  {a[:60]}  ->  {b[:60]}")

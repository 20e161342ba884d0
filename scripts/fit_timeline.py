"""Critical path of the LAST development fit in a rocprofv3 kernel trace of bench.py: per queue,
the first start / last end (ms from the fit's first kernel) and busy time of each kernel family,
and the idle gaps of the union of queues."""
import csv
import re
import sys
from collections import OrderedDict

rows = list(csv.DictReader(open(sys.argv[1])))
ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "?"))
            for r in rows)
starts = [i for i, k in enumerate(ks) if "knn_donor" in k[2]]
first = starts[-2] if len(starts) >= 2 else starts[0]
fit = ks[first:]
t0 = fit[0][0]


def short(n):
    n = re.sub(r"\(.*", "", n).replace("void ", "").replace("hfens::", "")
    return n[:44]


agg = OrderedDict()
for s, e, n, q in fit:
    k = (short(n), q)
    a = agg.setdefault(k, [s, e, 0, 0])
    a[1] = max(a[1], e)
    a[2] += 1
    a[3] += e - s
print(f"fit window {(fit[-1][1] - t0) / 1e6:.2f} ms, {len(fit)} kernels")
for (n, q), (s, e, c, t) in agg.items():
    if t > 100_000:
        print(f"{n:46s} q{q:>3} {(s - t0) / 1e6:7.2f} → {(e - t0) / 1e6:7.2f} ms  n={c:4d} busy {t / 1e6:6.2f} ms")
busy_end, idle = t0, 0
for s, e, n, q in fit:
    if s > busy_end:
        idle += s - busy_end
        if s - busy_end > 200_000:
            print(f"  idle {(s - busy_end) / 1e3:7.1f} us at {(busy_end - t0) / 1e6:6.2f} ms before {short(n)} (q{q})")
    busy_end = max(busy_end, e)
print(f"GPU idle inside the fit: {idle / 1e6:.2f} ms")

"""Per-fit GPU timeline from a rocprofv3 kernel-trace CSV: for the LAST development fit of a
bench run, kernels in start order with their queue, offset from the fit's first kernel and
duration, plus the idle gaps of the union of all queues (where the GPU did nothing).

    python scripts/timeline.py <kernel_trace.csv> [first-kernel-substring]
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    marker = sys.argv[2] if len(sys.argv) > 2 else "knn_donor_kernel"
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:70],
                  r.get("Queue_Id", r.get("Stream_Id", "?"))) for r in rows))
    starts = [i for i, k in enumerate(ks) if marker in k[2]]
    # each fit images two KNN launches (development rows, then held-out rows): the fit starts at
    # the second-to-last pair's first launch
    first = starts[-4] if len(starts) >= 4 else starts[0]
    last_fit = ks[first:]
    t0 = last_fit[0][0]
    agg = defaultdict(lambda: [0, 0.0])
    for s, e, n, q in last_fit:
        agg[(n, q)][0] += 1
        agg[(n, q)][1] += (e - s) / 1e3
    print(f"fit window: {(last_fit[-1][1] - t0) / 1e6:.2f} ms, {len(last_fit)} kernels")
    print("\n== kernels by total time (us) ==")
    for (n, q), (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:30]:
        print(f"{t:10.1f} {c:5d}  q{q}  {n}")
    print("\n== idle gaps > 100 us (union of queues) ==")
    busy_end = t0
    for s, e, n, q in last_fit:
        if s - busy_end > 100_000:
            print(f"  at {(busy_end - t0) / 1e6:7.2f} ms: idle {(s - busy_end) / 1e3:8.1f} us before {n} (q{q})")
        busy_end = max(busy_end, e)
    print("\n== long kernels (> 300 us) ==")
    for s, e, n, q in last_fit:
        if e - s > 300_000:
            print(f"  {(s - t0) / 1e6:7.2f} -> {(e - t0) / 1e6:7.2f} ms  q{q}  {n}")




def queue_activity(path, marker="knn_donor_kernel", gap_us=200.0):
    """Per queue: busy intervals of the FIRST fit in the window (merged across gaps < gap_us)."""
    rows = list(csv.DictReader(open(path)))
    ks = sorted(((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"][:60],
                  r.get("Queue_Id", r.get("Stream_Id", "?"))) for r in rows))
    starts = [i for i, k in enumerate(ks) if marker in k[2]]
    first = starts[-4] if len(starts) >= 4 else starts[0]
    end = starts[-2] if len(starts) >= 4 else len(ks)
    fit = ks[first:end]
    t0 = fit[0][0]
    byq = defaultdict(list)
    for k in fit:
        byq[k[3]].append(k)
    for q, kk in sorted(byq.items()):
        print(f"\n== queue {q}: {len(kk)} kernels ==")
        cur = None
        for s, e, n, _ in kk:
            if cur and s - cur[1] < gap_us * 1e3:
                cur[1] = max(cur[1], e)
                cur[2] += 1
                cur[4] = n
            else:
                if cur:
                    print(f"  {(cur[0] - t0) / 1e6:7.2f} -> {(cur[1] - t0) / 1e6:7.2f} ms  {cur[2]:4d} kernels  {cur[3]} .. {cur[4]}")
                cur = [s, e, 1, n, n]
        print(f"  {(cur[0] - t0) / 1e6:7.2f} -> {(cur[1] - t0) / 1e6:7.2f} ms  {cur[2]:4d} kernels  {cur[3]} .. {cur[4]}")


if len(sys.argv) > 3 and sys.argv[3] == "queues":
    queue_activity(sys.argv[1], sys.argv[2])


if __name__ == "__main__" and not (len(sys.argv) > 3 and sys.argv[3] == "queues"):
    main()

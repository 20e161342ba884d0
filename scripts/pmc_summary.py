"""Aggregate a rocprofv3 --pmc counter_collection.csv per kernel (sum of each counter over its
dispatches) into a small CSV; the raw per-dispatch file can be tens of MB."""
import collections
import csv
import sys


def main(src, dst, match=""):
    tot = collections.defaultdict(lambda: collections.defaultdict(float))
    calls = collections.Counter()
    seen = set()
    with open(src) as f:
        for r in csv.DictReader(f):
            name = r["Kernel_Name"]
            if match and match not in name:
                continue
            key = (r["Dispatch_Id"], r["Counter_Name"])
            tot[name][r["Counter_Name"]] += float(r["Counter_Value"])
            if r["Dispatch_Id"] not in seen:
                seen.add(r["Dispatch_Id"])
                calls[name] += 1
            del key
    names = sorted({c for d in tot.values() for c in d})
    with open(dst, "w") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "dispatches"] + names)
        for k in sorted(tot, key=lambda k: -calls[k]):
            w.writerow([k[:120], calls[k]] + [f"{tot[k].get(c, 0):.0f}" for c in names])


if __name__ == "__main__":
    main(*sys.argv[1:])

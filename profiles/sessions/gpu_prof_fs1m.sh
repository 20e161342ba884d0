#!/bin/bash
# Kernel-time totals of one 1M-row full development fit (BASELINE config 3), top kernels only.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/proffs
rm -rf $D && mkdir -p $D
timeout -k 10 900 rocprofv3 --kernel-trace --stats --output-format csv -d $D/raw -o fs -- python3 bench.py --rows 1000000 --steps 1 --warmup 0 > $D/log.txt 2>&1 || { tail -20 $D/log.txt; exit 1; }
f=$(find $D/raw -name "*kernel_stats.csv" | head -1)
python3 - "$f" > $D/top.txt <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e9:.2f} s")
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:30]:
    print(f'{float(r["TotalDurationNs"])/1e6:10.1f} ms {int(r["Calls"]):7d} {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:110]}')
PY
cp $f $D/stats.csv
find $D/raw -name "*kernel_trace.csv" -delete
cat $D/top.txt

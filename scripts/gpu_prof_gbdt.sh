#!/bin/bash
# Kernel-time breakdown of BASELINE config 3-GBC / config 5 benches (rocprofv3 kernel trace + stats).
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/profgb
mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/gbdt -o run --output-format csv -- python3 bench.py --config ${CFG:-gbdt} --steps 3 --warmup 1 ${EXTRA} > $D/log.txt 2>&1 || { echo "rocprof failed"; tail -20 $D/log.txt; exit 1; }
f=$(find $D/gbdt -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print("total kernel ms", round(tot / 1e6, 2))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:15]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.3f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:9.2f} us  {r["Name"][:90]}')
PY
tail -1 $D/log.txt

#!/bin/bash
# round 4: kernel stats of the headline bench after the Platt / sign changes
set -o pipefail
D=gpurun_out/r4u
mkdir -p $D
R=$PWD
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o hb --output-format csv -- python bench.py --steps 5 --warmup 2 > $D/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $D/prof.log; exit 1; }
f=$(find $D/prof -name "*kernel_stats.csv" | head -1)
cp $f $D/kernel_stats.csv
python - <<'PY'
import csv
r = list(csv.reader(open("gpurun_out/r4u/kernel_stats.csv")))
for x in r[1:25]:
    print(x[0][:60], x[1], round(float(x[3]) / 1e3, 1), "us avg", round(float(x[2]) / 1e6, 2), "ms", round(float(x[5]) / 1e3, 1), round(float(x[6]) / 1e3, 1))
PY
f=$(find $D/prof -name "*kernel_trace.csv" | head -1)
python - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in rows:
    n = r["Kernel_Name"]
    if "platt" in n or "svm_dec_batch" in n or "svc_oof" in n or "logreg_fused" in n:
        print(n[:40], (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
PY

#!/bin/bash
# Kernel statistics + GPU idle gaps of one low-rank SVC interior-point solve (rocprofv3 kernel trace).
#   bash scripts/gpu_ipm_prof.sh [ROWS] [LANDMARKS]
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
D=gpurun_out/ipmprof
rm -rf $D && mkdir -p $D
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $D/raw -o ipm -- python3 scripts/ipm_probe.py ${1:-1000000} ${2:-512} ipm-only > $D/probe.log 2>&1 \
  || { tail -20 $D/probe.log; exit 1; }
grep -v amdgpu.ids $D/probe.log | grep -v rocprofv3 | grep -v output_stream
f=$(find $D/raw -name "*kernel_stats.csv" | head -1)
t=$(find $D/raw -name "*kernel_trace.csv" | head -1)
python3 scripts/gap_report.py "$t" chol_spd > $D/gaps.txt && cat $D/gaps.txt
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
tot = sum(float(r["TotalDurationNs"]) for r in rows)
print(f"total kernel time {tot/1e6:.1f} ms")
for r in rows[:20]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d} {float(r["Percentage"]):6.2f}%  {r["Name"][:100]}')
PY
cp $f $D/ipm_kernel_stats.csv
rm -rf $D/raw

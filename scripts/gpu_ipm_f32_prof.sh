#!/bin/bash
# Kernel stats of the IPM probe (f64 map then f32-rounded map), to compare the skinny-pass kernels.
set -o pipefail
export TMPDIR=/tmp
D=gpurun_out/ipmf32prof
rm -rf $D && mkdir -p $D
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $D/raw -o ipm -- python3 scripts/probes/ipm_probe.py 1000000 512 ipm-only ${IPM_MAPS:-both} > $D/probe.log 2>&1 \
  || { tail -20 $D/probe.log; exit 1; }
grep "ipm solve" $D/probe.log
f=$(find $D/raw -name "*kernel_stats.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
for r in rows[:22]:
    print(f'{float(r["TotalDurationNs"])/1e6:9.2f} ms {int(r["Calls"]):6d} calls {float(r["AverageNs"])/1e3:9.1f} us  {r["Name"][:100]}')
PY

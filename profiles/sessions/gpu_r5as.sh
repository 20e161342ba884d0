#!/bin/bash
# Round 5: kernel statistics of the 1M-row imputation (matrix-core filter default).
set -o pipefail
O=gpurun_out/r5as
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 scripts/probes/knn_impute_scale.py 1000000 auto > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
grep -v amdgpu.ids $O/prof.log | tail -3
python3 - $O <<'PY'
import csv, sys
O = sys.argv[1]
r = list(csv.DictReader(open(f"{O}/prof/run_kernel_stats.csv")))
for x in r[:14]:
    print(f"{int(x['TotalDurationNs'])/1e6:9.2f} ms {int(x['Calls']):6d}  {x['Name'][:100]}")
PY
rm -f $O/prof/run_kernel_trace.csv

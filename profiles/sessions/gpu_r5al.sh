#!/bin/bash
# Round 5: config-3 (1M rows) kernel statistics — device busy time vs the fit's wall clock.
set -o pipefail
O=gpurun_out/r5al
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --rows 1000000 --steps 1 --warmup 0 > $O/bench.json 2> $O/bench.err || { echo "prof failed"; tail -20 $O/bench.err; exit 1; }
python3 - $O <<'PY'
import csv, sys, json
O = sys.argv[1]
r = list(csv.DictReader(open(f"{O}/prof/run_kernel_stats.csv")))
tot = sum(int(x['TotalDurationNs']) for x in r)
print("kernels total ms", tot / 1e6)
for x in r[:25]:
    print(f"{int(x['TotalDurationNs'])/1e6:9.1f} ms {int(x['Calls']):7d}  {x['Name'][:110]}")
t = list(csv.DictReader(open(f"{O}/prof/run_kernel_trace.csv")))
iv = sorted((int(x['Start_Timestamp']), int(x['End_Timestamp'])) for x in t)
busy, cur_s, cur_e = 0, None, None
for s, e in iv:
    if cur_e is None or s > cur_e:
        if cur_e is not None: busy += cur_e - cur_s
        cur_s, cur_e = s, e
    else:
        cur_e = max(cur_e, e)
busy += cur_e - cur_s
print("union busy ms", busy / 1e6, "span ms", (iv[-1][1] - iv[0][0]) / 1e6)
PY
tail -1 $O/bench.json | cut -c1-300

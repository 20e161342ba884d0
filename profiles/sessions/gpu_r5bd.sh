#!/bin/bash
# Round 5: headline kernel statistics (rocprofv3 --kernel-trace --stats), summary for profiles/.
set -o pipefail
O=gpurun_out/r5bd
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 10 --warmup 3 > $O/bench.json 2> $O/bench.err || { echo "prof failed"; tail -20 $O/bench.err; exit 1; }
python3 - $O <<'PY'
import csv, sys, json
O = sys.argv[1]
r = list(csv.DictReader(open(f"{O}/prof/run_kernel_stats.csv")))
tot = sum(int(x['TotalDurationNs']) for x in r)
d = json.loads(open(f"{O}/bench.json").read().strip().splitlines()[-1])
lines = [f"# Headline kernel statistics (round 5, `bench.py --steps 10 --warmup 3` under rocprofv3 --kernel-trace --stats)", "",
         f"bench under the profiler: {d['ms_per_step']} ms / fit; 13 fits in the process (3 warmup + 10 timed); kernel time summed over streams {tot/1e6:.1f} ms", "",
         "| kernel | calls | total ms | avg µs | % |", "|---|---:|---:|---:|---:|"]
for x in r[:30]:
    nm = x['Name'].split('(')[0].replace('|', '/')[:90]
    lines.append(f"| `{nm}` | {int(x['Calls'])} | {int(x['TotalDurationNs'])/1e6:.2f} | {float(x['AverageNs'])/1e3:.1f} | {float(x['Percentage']):.1f} |")
open(f"{O}/headline_kernel_stats.md", "w").write("\n".join(lines) + "\n")
print("\n".join(lines[:16]))
PY
rm -f $O/prof/run_kernel_trace.csv

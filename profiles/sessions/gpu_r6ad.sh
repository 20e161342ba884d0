#!/bin/bash
# Round 6: kernel stats of the headline (rocprofv3 --kernel-trace --stats), 5 timed steps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r6ad
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 3 > $O/bench.json 2> $O/prof.err || { echo "prof failed"; tail -20 $O/prof.err; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); echo "$f"; head -25 "$f" | cut -c1-220

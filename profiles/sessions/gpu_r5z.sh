#!/bin/bash
# Round 5: kernel statistics of the headline fit (current code) — 5 timed fits.
set -o pipefail
O=gpurun_out/r5z
mkdir -p $O
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/ks -o ks --output-format csv -- python3 bench.py --steps 5 --warmup 2 > $O/ks.log 2>&1 || { echo "ks failed"; tail -5 $O/ks.log; exit 1; }
f=$(find $O/ks -name "*kernel_stats.csv" | head -1); echo "stats: $f"; cp "$f" $O/headline_kernel_stats.csv
t=$(find $O/ks -name "*kernel_trace.csv" | head -1); cp "$t" $O/headline_kernel_trace.csv
head -30 $O/headline_kernel_stats.csv | cut -c1-220
rm -rf $O/ks

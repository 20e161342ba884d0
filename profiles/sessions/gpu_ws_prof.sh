#!/bin/bash
# Working-set SMO: per-problem rounds/pairs/phase cycles, then a kernel-time profile of the bench.
set -o pipefail
D=gpurun_out/wsprof
mkdir -p $D
HFENS_CONCURRENT_BASES=0 timeout -k 10 300 python scripts/ws_stats.py > $D/ws_stats.log 2>&1 || { echo "ws_stats failed"; tail -30 $D/ws_stats.log; exit 1; }
grep -v amdgpu.ids $D/ws_stats.log
export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $D/prof -o bench --output-format csv -- python bench.py --steps 3 --warmup 1 > $D/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $D/prof.log; exit 1; }
f=$(find $D/prof -name "*kernel_stats.csv" | head -1); echo "$f"; head -25 "$f" | cut -d, -f1-8

#!/bin/bash
# Round 5: where the 1M-row imputation's time goes (MFMA vs packed-FMA filter, kernel stats).
set -o pipefail
O=gpurun_out/r5ag
mkdir -p $O
true
true
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 scripts/probes/knn_impute_scale.py 1000000 1 > $O/prof.log 2>&1 || { echo "prof failed"; tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name '*kernel_stats.csv' | head -1); head -14 "$f" | cut -c1-160

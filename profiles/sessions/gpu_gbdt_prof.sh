#!/bin/bash
# GBDT-only 1M x 40 (cfg 3 analog): stage vs launch path, kernel stats of each.
set -o pipefail
D=gpurun_out/gbdtprof
mkdir -p $D
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for path in stage launch; do
  HFENS_GBDT_STUMPS=$path timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/$path -o g --output-format csv -- python3 bench.py --config gbdt --steps 3 --warmup 1 > $D/$path.log 2>&1 || { echo "$path failed"; tail -20 $D/$path.log; exit 1; }
  grep metric $D/$path.log | cut -c1-200
  f=$(find $D/$path -name "*kernel_stats.csv" | head -1)
  head -6 $f | cut -d, -f1-5 | cut -c1-160
done

#!/bin/bash
# Round 6: step outliers back to back (as bench.py times them), config 4 / 5 / gbdt records on the current tree.
set -o pipefail
O=gpurun_out/r6n
mkdir -p $O
SYNC=0 timeout -k 10 300 python scripts/probes/step_outliers.py 100 > $O/outliers_nosync.log 2>&1 && tail -1 $O/outliers_nosync.log | cut -c1-2500
timeout -k 10 300 python bench.py --config infer --steps 10 --warmup 3 > $O/infer.json 2> $O/infer.err || { echo "infer failed"; tail -20 $O/infer.err; exit 1; }
tail -1 $O/infer.json | cut -c1-600
timeout -k 10 300 python bench.py --config gbdt --steps 10 --warmup 3 > $O/gbdt.json 2> $O/gbdt.err || { echo "gbdt failed"; tail -20 $O/gbdt.err; exit 1; }
tail -1 $O/gbdt.json | cut -c1-600
timeout -k 10 400 python bench.py --config deep --steps 5 --warmup 2 > $O/deep.json 2> $O/deep.err || { echo "deep failed"; tail -20 $O/deep.err; exit 1; }
tail -1 $O/deep.json | cut -c1-900

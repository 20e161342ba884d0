#!/bin/bash
set -o pipefail
D=gpurun_out/gbmarks
mkdir -p $D
timeout -k 10 300 python scripts/probes/gbdt_fit_marks.py > $D/marks.log 2>&1 || { echo "marks failed"; tail -30 $D/marks.log; exit 1; }
grep "^\[" $D/marks.log

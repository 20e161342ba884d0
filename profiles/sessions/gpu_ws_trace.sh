#!/bin/bash
# Kernel trace of the headline fit with sequential bases: per-round durations of the working-set
# SMO kernels (lockstep of the 36 problems) and the logistic-regression kernel.
set -o pipefail
D=gpurun_out/wstrace
rm -rf $D; mkdir -p $D
export TMPDIR=/tmp
HFENS_CONCURRENT_BASES=0 timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/raw -o tr -- python scripts/ws_stats.py > $D/run.log 2>&1 || { echo "trace failed"; tail -20 $D/run.log; exit 1; }
f=$(find $D/raw -name "*kernel_trace.csv" | head -1)
python scripts/probes/ws_trace_report.py "$f" > $D/report.txt && cat $D/report.txt
rm -rf $D/raw

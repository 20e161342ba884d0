#!/bin/bash
set -o pipefail
O=gpurun_out/r6f
mkdir -p $O
timeout -k 10 200 python scripts/probes/host_window_r6.py > $O/host_window.log 2>&1 || { echo "probe failed"; tail -30 $O/host_window.log; exit 1; }
grep "====\|wall ms" $O/host_window.log

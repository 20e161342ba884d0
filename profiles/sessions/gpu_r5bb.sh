#!/bin/bash
# Round 5: interior-point starting point sweep at 300k rows.
set -o pipefail
O=gpurun_out/r5bb
mkdir -p $O
timeout -k 10 500 python -u scripts/probes/ipm_start_sweep.py 300000 > $O/sweep.log 2>&1 || { echo "probe failed"; tail -20 $O/sweep.log; exit 1; }
grep -v amdgpu.ids $O/sweep.log

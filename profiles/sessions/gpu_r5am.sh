#!/bin/bash
# Round 5: r × r factor latency under contention (stream priority).
set -o pipefail
O=gpurun_out/r5am
mkdir -p $O
timeout -k 10 300 python -u scripts/probes/chol_contention.py > $O/chol.log 2>&1 || { echo "probe failed"; tail -20 $O/chol.log; exit 1; }
grep -v amdgpu.ids $O/chol.log

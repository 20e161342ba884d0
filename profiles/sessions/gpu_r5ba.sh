#!/bin/bash
# Round 5: interior-point convergence trajectory at 300k rows.
set -o pipefail
O=gpurun_out/r5ba
mkdir -p $O
HFENS_IPM_DEBUG=1 timeout -k 10 300 python -u scripts/probes/ipm_trajectory.py 300000 > $O/traj.log 2>&1 || { echo "probe failed"; tail -20 $O/traj.log; exit 1; }
grep -v amdgpu.ids $O/traj.log | cut -c1-220

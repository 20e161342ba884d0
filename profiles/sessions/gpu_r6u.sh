#!/bin/bash
# Round 6: the interior point's trajectory at 1M rows (gap / residuals / steps per iteration).
set -o pipefail
O=gpurun_out/r6u
mkdir -p $O
HFENS_IPM_DEBUG=1 timeout -k 10 300 python scripts/probes/ipm_trajectory.py 1000000 > $O/traj_1m.log 2>&1 || { echo "traj failed"; tail -20 $O/traj_1m.log; exit 1; }
grep -c "\[ipm\] it" $O/traj_1m.log; tail -3 $O/traj_1m.log

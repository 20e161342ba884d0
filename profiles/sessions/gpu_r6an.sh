#!/bin/bash
# Round 6: config-3 interior point — Gondzio correctors per iteration (2 = default, 4, 6) on one 1M problem.
set -o pipefail
O=gpurun_out/r6an
mkdir -p $O
for k in 2 4 6 1; do
  HFENS_IPM_CORRECTORS=$k REPS=2 timeout -k 10 240 python scripts/probes/ipm_trajectory.py 1000000 > $O/traj_c$k.log 2>&1 || { echo "traj $k failed"; tail -20 $O/traj_c$k.log; exit 1; }
  tail -1 $O/traj_c$k.log
done

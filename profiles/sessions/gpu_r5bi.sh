#!/bin/bash
# Round 5: host profile of the SVC prelaunch in the headline step.
set -o pipefail
O=gpurun_out/r5bi
mkdir -p $O
timeout -k 10 300 python -u scripts/probes/host_profile_svc.py > $O/prof.log 2>&1 || { echo "probe failed"; tail -20 $O/prof.log; exit 1; }
grep -v amdgpu.ids $O/prof.log | head -120

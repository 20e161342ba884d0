#!/bin/bash
set -o pipefail
O=gpurun_out/r5w
mkdir -p $O
timeout -k 10 300 python scripts/probes/gbdt_stage_phases.py > $O/phases.log 2>&1 || { echo "phases failed"; tail -20 $O/phases.log; exit 1; }
grep -v amdgpu.ids $O/phases.log
PROBE_ROWS=125000 timeout -k 10 300 python scripts/probes/gbdt_stage_phases.py > $O/phases_125k.log 2>&1 || { echo "phases failed"; tail -20 $O/phases_125k.log; exit 1; }
grep -v amdgpu.ids $O/phases_125k.log

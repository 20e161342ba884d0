#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
HFENS_PROFILE_SMO=1 timeout -k 10 300 python scripts/ws_diag.py exact > gpurun_out/smo_prof.log 2>&1 || { tail -20 gpurun_out/smo_prof.log; exit 1; }
grep -v amdgpu.ids gpurun_out/smo_prof.log

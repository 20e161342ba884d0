#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
WS_DIAG_ROWS=20000 WS_DIAG_REPS=1 timeout -k 10 400 python scripts/ws_diag.py ws:0.1 exact > gpurun_out/ws_diag20k.log 2>&1 || { tail -20 gpurun_out/ws_diag20k.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ws_diag20k.log

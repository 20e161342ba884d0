#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_svm_ws_gpu.py -x -q > gpurun_out/pytest_ws.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_ws.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_ws.log; exit 1; }
timeout -k 10 300 python scripts/ws_diag.py exact ws:0.1 > gpurun_out/ws_diag.log 2>&1 || { tail -20 gpurun_out/ws_diag.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ws_diag.log
bash scripts/gpu_ws4.sh > /dev/null

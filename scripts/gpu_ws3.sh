#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_svm_ws_gpu.py -x -q > gpurun_out/pytest_ws.log 2>&1; rc=$?
tail -30 gpurun_out/pytest_ws.log
[ $rc -eq 0 ] || exit 1
bash scripts/gpu_ws2.sh

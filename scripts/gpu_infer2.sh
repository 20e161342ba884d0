#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_stack_infer.py -m gpu -x -q > gpurun_out/pytest_infer.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_infer.log; exit 1; }
tail -2 gpurun_out/pytest_infer.log
timeout -k 10 600 python scripts/infer_tune.py > gpurun_out/infer_tune.log 2>&1 || { echo "tune failed"; tail -30 gpurun_out/infer_tune.log; exit 1; }
cat gpurun_out/infer_tune.log

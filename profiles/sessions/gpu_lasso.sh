#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_prep_gpu.py -x -q > gpurun_out/pytest_prep.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_prep.log
[ $rc -eq 0 ] || { tail -30 gpurun_out/pytest_prep.log; exit 1; }
bash scripts/gpu_prof_bench.sh

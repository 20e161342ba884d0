#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_svm_ws_gpu.py -x -q > gpurun_out/pytest_ws.log 2>&1; rc=$?
tail -40 gpurun_out/pytest_ws.log
[ $rc -eq 0 ] || exit 1
HFENS_SVM_SOLVER=ws timeout -k 10 300 python bench.py --steps 3 --warmup 1 --timings > gpurun_out/bench_ws.json 2> gpurun_out/bench_ws.err || { echo "bench ws failed"; tail -30 gpurun_out/bench_ws.err; exit 1; }
grep -v amdgpu.ids gpurun_out/bench_ws.err; cat gpurun_out/bench_ws.json

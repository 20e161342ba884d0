#!/bin/bash
# quick check: SVC/stack GPU tests, bench with host marks
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_train_gpu.py tests/test_checkpoint.py tests/test_svm_ws_gpu.py tests/test_robustness.py -x -q -m gpu > gpurun_out/pytest_quick.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_quick.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_quick.log; exit 1; }
HFENS_TRACE_HOST=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 --timings > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
grep "\[host\]" gpurun_out/bench.err | tail -3; grep -v "amdgpu.ids\|\[host\]" gpurun_out/bench.err; cat gpurun_out/bench.json

#!/bin/bash
# Fused-inference session: numerics tests, 100M-row infer bench, kernel profile.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_stack_infer.py tests/test_infer_gpu.py -m gpu -x -q > gpurun_out/pytest_infer.log 2>&1 || { echo "pytest failed rc=$?"; tail -40 gpurun_out/pytest_infer.log; exit 1; }
tail -3 gpurun_out/pytest_infer.log
timeout -k 10 300 python bench.py --config infer --steps 5 --warmup 1 > gpurun_out/bench_infer.json 2> gpurun_out/bench_infer.err || { echo "bench failed"; tail -30 gpurun_out/bench_infer.err; exit 1; }
cat gpurun_out/bench_infer.json
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_infer -o infer --output-format csv -- python bench.py --config infer --rows 20000000 --steps 2 --warmup 1 > gpurun_out/prof_infer.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_infer.log; exit 1; }
find gpurun_out/prof_infer -name "*stats*"

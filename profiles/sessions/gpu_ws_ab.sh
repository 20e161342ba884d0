#!/bin/bash
# Working-set SMO (svm_ws.hip, q = 1024): numerics tests, then the driver's bench with the
# working-set solver (default) and with the exact pair sequence.  Stop at the first failure.
set -o pipefail
D=gpurun_out/wsab
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_svm_ws_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $D/pytest.log; exit 1; }
tail -4 $D/pytest.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --timings > $D/bench_ws.json 2> $D/bench_ws.err || { echo "bench ws failed"; tail -30 $D/bench_ws.err; exit 1; }
cat $D/bench_ws.json; grep -v amdgpu.ids $D/bench_ws.err | tail -20
HFENS_SVM_SOLVER=exact timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $D/bench_exact.json 2> $D/bench_exact.err || { echo "bench exact failed"; tail -30 $D/bench_exact.err; exit 1; }
cat $D/bench_exact.json

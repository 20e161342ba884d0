#!/bin/bash
# Round 3: fused interior-point kernels — tests, kernel stats at 1M rows, config 3 warm.
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_linalg_gpu.py tests/test_svc_lowrank.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3i_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r3i_pytest.log; exit 1; }
tail -2 gpurun_out/r3i_pytest.log
bash scripts/probes/gpu_r3h.sh

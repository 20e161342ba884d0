#!/bin/bash
# Round 3: skinny passes (flat Φᵀv, contiguous Φw): launch-shape probe, low-rank tests, IPM kernel
# stats at 1M rows and config 3 warm.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python3 -u scripts/probes/skinny_probe.py > gpurun_out/skinny_probe.log 2>&1 || { echo "probe failed"; tail -20 gpurun_out/skinny_probe.log; exit 1; }
grep -v amdgpu.ids gpurun_out/skinny_probe.log
timeout -k 10 400 python -u -m pytest tests/test_linalg_gpu.py tests/test_svc_lowrank.py tests/test_train_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3l_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r3l_pytest.log; exit 1; }
tail -2 gpurun_out/r3l_pytest.log
bash scripts/probes/gpu_r3h.sh

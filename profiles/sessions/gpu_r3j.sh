#!/bin/bash
# Round 3: fused IPM tails + KNN tests, IPM kernel stats, config 3 warm, KNN rate.
set -o pipefail
timeout -k 10 400 python -u -m pytest tests/test_linalg_gpu.py tests/test_svc_lowrank.py tests/test_prep_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3j_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r3j_pytest.log; exit 1; }
tail -2 gpurun_out/r3j_pytest.log
timeout -k 10 300 python3 scripts/probes/knn_probe.py 300000 > gpurun_out/r3j_knn.log 2>&1 || { echo "knn failed"; tail -20 gpurun_out/r3j_knn.log; exit 1; }
grep rows gpurun_out/r3j_knn.log
bash scripts/probes/gpu_r3h.sh

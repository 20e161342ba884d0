#!/bin/bash
# Round 6 (end): low-rank SVC tests with three fits solved at a time (the new default).
set -o pipefail
O=gpurun_out/r6ce
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_svc_scale_gpu.py tests/test_linalg_gpu.py tests/test_nystrom_gpu.py tests/test_svc_lowrank.py tests/test_train_gpu.py -q --timeout 300 --timeout-method thread -p no:cacheprovider -m gpu > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log

#!/bin/bash
set -o pipefail
D=gpurun_out/lr
mkdir -p $D
timeout -k 10 300 python3 -u -m pytest tests/test_train_gpu.py -k "logreg" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1 \
  || { echo "pytest failed"; tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
bash scripts/gpu_quick.sh

#!/bin/bash
# Round 5: the KNN donor filter on the bf16 matrix cores — equality with the packed-FMA kernel, speed.
set -o pipefail
O=gpurun_out/r5ac
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_prep_gpu.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider -k "mfma_filter" > $O/pytest_mfma.log 2>&1 || { echo "pytest mfma failed"; tail -40 $O/pytest_mfma.log; exit 1; }
tail -2 $O/pytest_mfma.log
timeout -k 10 300 python scripts/probes/knn_mfma_probe.py 10000 100000 300000 > $O/probe.log 2>&1 || { echo "probe failed"; tail -20 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log
HFENS_KNN_MFMA=1 timeout -k 10 600 python -u -m pytest tests/test_prep_gpu.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_prep.log 2>&1 || { echo "pytest prep failed"; tail -40 $O/pytest_prep.log; exit 1; }
tail -2 $O/pytest_prep.log

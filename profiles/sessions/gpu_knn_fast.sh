#!/bin/bash
# KNN: the fast-pass kernel against the exact direct kernel (same donors, tested) and their rates.
set -o pipefail
D=gpurun_out/knnfast
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_prep_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider -k "knn" > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
for k in direct fast; do
  HFENS_KNN_KERNEL=$k timeout -k 10 300 python3 scripts/probes/knn_probe.py 100000 300000 > $D/probe_$k.log 2>&1 || { echo "probe $k failed"; tail -20 $D/probe_$k.log; exit 1; }
  echo "== $k"; grep rows $D/probe_$k.log
done

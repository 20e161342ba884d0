#!/bin/bash
# round 4: persistent GBDT stage loop — bit-identity tests, per-stage probe
set -o pipefail
D=gpurun_out/r4x
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "gbdt" > $D/pytest_gbdt.log 2>&1 || { echo "pytest failed"; tail -40 $D/pytest_gbdt.log; exit 1; }
tail -2 $D/pytest_gbdt.log
timeout -k 10 300 python -u scripts/probes/gbdt_persist_probe.py > $D/persist_probe.log 2>&1 || { echo "probe failed"; tail -30 $D/persist_probe.log; exit 1; }
grep -v "^{" $D/persist_probe.log | tail -10

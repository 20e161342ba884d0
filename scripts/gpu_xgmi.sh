#!/bin/bash
# Peer-memory (IPC / xGMI) GBDT stage reduction: multi-process tests on one card, then the
# existing stage-path tests.
set -o pipefail
D=gpurun_out/xgmi
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_train_gpu.py -x -v -k "data_parallel or xgmi or graph" --timeout 240 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $D/pytest.log; exit 1; }
tail -12 $D/pytest.log
timeout -k 10 300 python scripts/probes/gbdt_shard_probe.py > $D/shard_probe.log 2>&1 || { echo "probe failed"; tail -30 $D/shard_probe.log; exit 1; }
grep -v amdgpu.ids $D/shard_probe.log | grep -v "^{"

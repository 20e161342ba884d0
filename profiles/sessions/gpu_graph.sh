#!/bin/bash
set -o pipefail
D=gpurun_out/graph
mkdir -p $D
timeout -k 10 300 python3 -u -m pytest tests/test_train_gpu.py -k "graph or stage or stump" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1 \
  || { echo "pytest failed"; tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
timeout -k 10 300 python3 -u scripts/stage_graph_overhead.py 125000 > $D/overhead.log 2>&1 || { echo "overhead failed"; tail -30 $D/overhead.log; exit 1; }
cat $D/overhead.log | grep -v amdgpu.ids

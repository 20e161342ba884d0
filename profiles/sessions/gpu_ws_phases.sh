#!/bin/bash
set -o pipefail
D=gpurun_out/wsph
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_svm_ws_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
HFENS_PROFILE_WS=1 HFENS_CONCURRENT_BASES=0 timeout -k 10 300 python scripts/ws_stats.py > $D/ws_stats.log 2>&1 || { echo "ws_stats failed"; tail -30 $D/ws_stats.log; exit 1; }
grep -v amdgpu.ids $D/ws_stats.log | tail -8
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -30 $D/bench.err; exit 1; }
cat $D/bench.json

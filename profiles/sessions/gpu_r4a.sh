#!/bin/bash
# round 4: K-cached working-set SMO (q = 256) — tests, per-problem stats, bench A/B against q = 1024
set -o pipefail
D=gpurun_out/r4a
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_svm_ws_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
HFENS_CONCURRENT_BASES=0 timeout -k 10 300 python scripts/ws_stats.py > $D/ws_stats.log 2>&1 || { echo "ws_stats failed"; tail -30 $D/ws_stats.log; exit 1; }
grep -v amdgpu.ids $D/ws_stats.log | tail -8
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $D/bench_kc.json 2> $D/bench_kc.err || { echo "bench failed"; tail -30 $D/bench_kc.err; exit 1; }
cat $D/bench_kc.json
HFENS_SVM_WS_KC=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $D/bench_q1024.json 2> $D/bench_q1024.err || { echo "bench failed"; tail -30 $D/bench_q1024.err; exit 1; }
cat $D/bench_q1024.json

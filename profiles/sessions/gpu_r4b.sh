#!/bin/bash
# round 4: K-cached SMO tests + bench A/B, then the large-problem candidate selection (40k test, crossover)
set -o pipefail
D=gpurun_out/r4b
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_svm_ws_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest_ws.log 2>&1 || { echo "pytest ws failed"; tail -40 $D/pytest_ws.log; exit 1; }
tail -3 $D/pytest_ws.log
HFENS_CONCURRENT_BASES=0 timeout -k 10 300 python scripts/ws_stats.py > $D/ws_stats.log 2>&1 || { echo "ws_stats failed"; tail -30 $D/ws_stats.log; exit 1; }
grep -v amdgpu.ids $D/ws_stats.log | tail -8
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $D/bench_kc.json 2> $D/bench_kc.err || { echo "bench failed"; tail -30 $D/bench_kc.err; exit 1; }
cat $D/bench_kc.json
HFENS_SVM_WS_KC=0 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $D/bench_q1024.json 2> $D/bench_q1024.err || { echo "bench failed"; tail -30 $D/bench_q1024.err; exit 1; }
cat $D/bench_q1024.json
timeout -k 10 300 python -u -m pytest tests/test_svc_scale_gpu.py -x -v --timeout 280 --timeout-method thread -p no:cacheprovider > $D/pytest_scale.log 2>&1 || { echo "pytest scale failed"; tail -40 $D/pytest_scale.log; exit 1; }
tail -3 $D/pytest_scale.log
timeout -k 10 400 python -u scripts/probes/svc_crossover.py 40000 100000 > $D/crossover.log 2>&1 || { echo "crossover failed"; tail -30 $D/crossover.log; exit 1; }
cat $D/crossover.log

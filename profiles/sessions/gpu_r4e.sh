#!/bin/bash
# round 4: q = 1024 solver with the simplified key computation (headline default again), K-cached
# forced for comparison, GPU tests of the SVC paths, crossover at 200k / 300k rows
set -o pipefail
D=gpurun_out/r4e
mkdir -p $D
timeout -k 10 500 python -u -m pytest tests/test_svm_ws_gpu.py tests/test_svc_scale_gpu.py tests/test_linalg_gpu.py -v --timeout 280 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1
rc=$?
tail -5 $D/pytest.log
# (test failures are recorded and the measurements still run; a timeout / crash stops here)
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc"; exit 1; fi
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -30 $D/bench.err; exit 1; }
cat $D/bench.json
HFENS_SVM_WS_KC=1 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $D/bench_kc.json 2> $D/bench_kc.err || { echo "bench failed"; tail -30 $D/bench_kc.err; exit 1; }
cat $D/bench_kc.json
HFENS_CONCURRENT_BASES=0 timeout -k 10 300 python scripts/ws_stats.py > $D/ws_stats.log 2>&1 || { echo "ws_stats failed"; tail -30 $D/ws_stats.log; exit 1; }
grep -v amdgpu.ids $D/ws_stats.log | tail -8
HFENS_IPM_GRAM=f64 timeout -k 10 200 python -u scripts/probes/ipm_probe.py 1000000 512 ipm-only f32-only > $D/ipm_f64.log 2>&1 || { echo "ipm f64 failed"; tail -20 $D/ipm_f64.log; exit 1; }
cat $D/ipm_f64.log
HFENS_IPM_GRAM=f32 timeout -k 10 200 python -u scripts/probes/ipm_probe.py 1000000 512 ipm-only f32-only > $D/ipm_f32.log 2>&1 || { echo "ipm f32 failed"; tail -20 $D/ipm_f32.log; exit 1; }
cat $D/ipm_f32.log
timeout -k 10 500 python -u scripts/probes/svc_crossover.py 200000 300000 > $D/crossover.log 2>&1 || { echo "crossover failed"; tail -30 $D/crossover.log; exit 1; }
cat $D/crossover.log

#!/bin/bash
# round 4: K-cached SMO phase stamps + bench A/B (graphs, q = 1024); large-problem crossover;
# f32-MFMA interior-point Gram (kernel tests, 1M-row IPM probe f32 vs f64)
set -o pipefail
D=gpurun_out/r4d
mkdir -p $D
HFENS_PROFILE_WS=1 HFENS_CONCURRENT_BASES=0 timeout -k 10 300 python scripts/ws_stats.py > $D/ws_stats_prof.log 2>&1 || { echo "ws_stats failed"; tail -30 $D/ws_stats_prof.log; exit 1; }
grep -v amdgpu.ids $D/ws_stats_prof.log | tail -7
timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $D/bench_kc.json 2> $D/bench_kc.err || { echo "bench failed"; tail -30 $D/bench_kc.err; exit 1; }
cat $D/bench_kc.json
HFENS_SVM_WS_GRAPH=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $D/bench_kc_nograph.json 2> $D/bench_kc_nograph.err || { echo "bench failed"; tail -30 $D/bench_kc_nograph.err; exit 1; }
cat $D/bench_kc_nograph.json
HFENS_SVM_WS_KC=0 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $D/bench_q1024.json 2> $D/bench_q1024.err || { echo "bench failed"; tail -30 $D/bench_q1024.err; exit 1; }
cat $D/bench_q1024.json
timeout -k 10 300 python -u scripts/probes/svc_crossover.py 40000 100000 > $D/crossover.log 2>&1 || { echo "crossover failed"; tail -30 $D/crossover.log; exit 1; }
cat $D/crossover.log
timeout -k 10 400 python -u -m pytest tests/test_linalg_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest_linalg.log 2>&1 || { echo "pytest linalg failed"; tail -40 $D/pytest_linalg.log; exit 1; }
tail -3 $D/pytest_linalg.log
HFENS_IPM_GRAM=f64 timeout -k 10 200 python -u scripts/probes/ipm_probe.py 1000000 512 ipm-only f32-only > $D/ipm_f64.log 2>&1 || { echo "ipm f64 failed"; tail -20 $D/ipm_f64.log; exit 1; }
cat $D/ipm_f64.log
HFENS_IPM_GRAM=f32 timeout -k 10 200 python -u scripts/probes/ipm_probe.py 1000000 512 ipm-only f32-only > $D/ipm_f32.log 2>&1 || { echo "ipm f32 failed"; tail -20 $D/ipm_f32.log; exit 1; }
cat $D/ipm_f32.log

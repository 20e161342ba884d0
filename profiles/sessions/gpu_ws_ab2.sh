#!/bin/bash
# WS inner solver: numerics tests, 256 vs 512 threads (sequential bases, per-pair cost), bench.
set -o pipefail
D=gpurun_out/wsab2
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_svm_ws_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for th in 256 512; do
  HFENS_SVM_WS_THREADS=$th HFENS_CONCURRENT_BASES=0 timeout -k 10 300 python scripts/ws_stats.py > $D/ws_$th.log 2>&1 || { echo "ws_stats $th failed"; tail -30 $D/ws_$th.log; exit 1; }
  echo "== threads $th"; grep "problem 35\|fit_svc" $D/ws_$th.log
  HFENS_SVM_WS_THREADS=$th timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $D/bench_$th.json 2> $D/bench_$th.err || { echo "bench failed"; tail -30 $D/bench_$th.err; exit 1; }
  python -c "import json;d=json.load(open('$D/bench_$th.json'));print('bench', d['ms_per_step'], d['config']['stage_seconds'], d['auroc'])"
done
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py -x -q -k "stage_plan or lowrank or svc" --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest2.log 2>&1 || { echo "pytest2 failed"; tail -40 $D/pytest2.log; exit 1; }
tail -1 $D/pytest2.log
timeout -k 10 400 python -u -m pytest tests/test_svc_lowrank.py tests/test_linalg_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest3.log 2>&1 || { echo "pytest3 failed"; tail -40 $D/pytest3.log; exit 1; }
tail -1 $D/pytest3.log

#!/bin/bash
set -o pipefail
D=gpurun_out/r4p
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_prep_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k knn > $D/pytest_knn.log 2>&1 || { echo "pytest knn failed"; tail -40 $D/pytest_knn.log; exit 1; }
tail -2 $D/pytest_knn.log
timeout -k 10 120 python -u scripts/probes/knn_refine_probe.py > $D/probe.log 2>&1 || { echo "probe failed"; tail -20 $D/probe.log; exit 1; }
grep rep $D/probe.log
for k in 1 0; do
  HFENS_KNN_EXACT=$k timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $D/bench_exact$k.json 2> $D/bench_exact$k.err || { echo "bench failed"; tail -30 $D/bench_exact$k.err; exit 1; }
  python -c "import json; d=json.loads(open('$D/bench_exact$k.json').read().strip().split('\n')[-1]); print('exact$k', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"
done

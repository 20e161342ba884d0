#!/bin/bash
# Working-set SMO: build-phase rewrite check + inner-pair cap sweep on the driver's bench.
set -o pipefail
D=gpurun_out/wscap
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_svm_ws_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
HFENS_CONCURRENT_BASES=0 timeout -k 10 300 python scripts/ws_stats.py > $D/ws.log 2>&1 || { echo "ws_stats failed"; tail -30 $D/ws.log; exit 1; }
grep "problem 35\|fit_svc" $D/ws.log
for cap in 4096 512 384 256; do
  HFENS_SVM_WS_INNER=$cap timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $D/bench_$cap.json 2>/dev/null || { echo "bench failed"; exit 1; }
  python -c "import json;d=json.load(open('$D/bench_$cap.json'));print('cap $cap', d['ms_per_step'], d['auroc'], d['diag']['svm'], d['diag']['step_ms_min_med_max'])"
done

#!/bin/bash
# WS inner-solver width A/B (256 vs 512 threads) and L1-LR member sweep.
set -o pipefail
D=gpurun_out/wslr
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_svm_ws_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for th in 256 512; do
  HFENS_SVM_WS_THREADS=$th HFENS_CONCURRENT_BASES=0 timeout -k 10 300 python scripts/ws_stats.py > $D/ws_$th.log 2>&1 || { echo "ws_stats $th failed"; tail -30 $D/ws_$th.log; exit 1; }
  echo "== threads $th"; grep "problem 35\|fit_svc" $D/ws_$th.log
done
for m in 0 1 4 8; do
  HFENS_LOGREG_MEMBERS=$m HFENS_CONCURRENT_BASES=0 timeout -k 10 300 python scripts/probes/lr_probe.py > $D/lr_$m.log 2>&1 || { echo "lr $m failed"; tail -30 $D/lr_$m.log; exit 1; }
  grep members $D/lr_$m.log
done

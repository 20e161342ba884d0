#!/bin/bash
# Standard GPU check: kernel/GPU tests, then the driver's exact bench command (twice: run-to-run
# spread), then smoke.  Each GPU step has its own limit; stop at the first failure.
set -o pipefail
D=gpurun_out/check
mkdir -p $D
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $D/pytest_gpu.log 2>&1 \
  || { echo "pytest failed rc=$?"; tail -40 $D/pytest_gpu.log; exit 1; }
tail -2 $D/pytest_gpu.log
for k in 1 2; do
  timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench$k.json 2> $D/bench$k.err \
    || { echo "bench failed"; tail -30 $D/bench$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench$k.json')); print('bench$k', d['ms_per_step'], d['config']['stage_seconds'], d['diag']['step_ms_min_med_max'], d['diag']['svm'])"
done
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke failed"; tail -30 $D/smoke.log; exit 1; }
tail -2 $D/smoke.log

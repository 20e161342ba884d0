#!/bin/bash
# Shared Platt-CV Grams: SMO exactness tests, then the driver's bench with sharing on and off.
set -o pipefail
D=gpurun_out/share
mkdir -p $D
timeout -k 10 600 python3 -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_train_gpu.py \
    -k "smo_shared_gram or smo_coop_matches" > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $D/pytest.log; exit 1; }
grep -E "passed|failed" $D/pytest.log | tail -2
for v in 1 0 1; do
  HFENS_SMO_SHARE_GRAM=$v timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench$v.json 2> $D/bench$v.err \
    || { echo "bench failed"; tail -30 $D/bench$v.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$D/bench$v.json').read().strip().splitlines()[-1]); print('share=$v', d['ms_per_step'], d['auroc'], d['diag']['step_ms_min_med_max'], d['diag']['svm'])"
done

#!/bin/bash
# Round 3: contraction pragmas honoured (-ffp-contract=fast-honor-pragmas): the full GPU suite,
# the headline, the KNN rate, interior-point kernel stats at 1M rows and config 3 warm.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > gpurun_out/r3k_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r3k_pytest.log; exit 1; }
tail -2 gpurun_out/r3k_pytest.log
timeout -k 10 300 python bench.py --steps 10 --warmup 3 --timings > gpurun_out/r3k_head.json 2> gpurun_out/r3k_head.err || { echo "bench failed"; tail -30 gpurun_out/r3k_head.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r3k_head.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['auroc'], d['diag'].get('step_ms_min_med_max'))"
timeout -k 10 300 python3 scripts/probes/knn_probe.py 300000 > gpurun_out/r3k_knn.log 2>&1 || { echo "knn failed"; tail -20 gpurun_out/r3k_knn.log; exit 1; }
grep rows gpurun_out/r3k_knn.log
bash scripts/probes/gpu_r3h.sh

#!/bin/bash
# Round 5: matrix-core KNN filter without a donor-range cap per split: tests, probe, 1M imputation, config 3.
set -o pipefail
O=gpurun_out/r5av
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_prep_gpu.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_prep.log 2>&1 || { echo "pytest prep failed"; tail -40 $O/pytest_prep.log; exit 1; }
tail -2 $O/pytest_prep.log
timeout -k 10 300 python scripts/probes/knn_mfma_probe.py 10000 50000 100000 300000 > $O/probe.log 2>&1 || { echo "probe failed"; tail -20 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log
timeout -k 10 300 python -u scripts/probes/knn_impute_scale.py 1000000 0,auto > $O/scale.log 2>&1 || { echo "scale failed"; tail -20 $O/scale.log; exit 1; }
grep -v amdgpu.ids $O/scale.log
timeout -k 10 900 python -u bench.py --rows 1000000 --steps 2 --warmup 1 > $O/fullstack_1m.json 2> $O/fullstack_1m.err || { echo "1m failed"; tail -20 $O/fullstack_1m.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/fullstack_1m.json').read().strip().splitlines()[-1]);print('1M', d['ms_per_step'], d['auroc'], d['diag'].get('step_ms_min_med_max'), d['config'].get('stage_seconds'))"

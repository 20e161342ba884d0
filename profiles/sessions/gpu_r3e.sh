#!/bin/bash
# Round 3: fp8 f8f6f4 forest + KNN fast pass (tests, rates), the headline, the dp rehearsal.
set -o pipefail
D=gpurun_out/r3e
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_forest_fp8_gpu.py tests/test_prep_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
for k in direct fast; do
  HFENS_KNN_KERNEL=$k timeout -k 10 300 python3 scripts/probes/knn_probe.py 100000 300000 > $D/knn_$k.log 2>&1 || { echo "probe $k failed"; tail -20 $D/knn_$k.log; exit 1; }
  echo "== $k"; grep rows $D/knn_$k.log
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $D/headline.json 2> $D/headline.err || { echo "headline failed"; tail -30 $D/headline.err; exit 1; }
python3 -c "import json; d=json.loads(open('$D/headline.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['auroc'], d['config']['stage_seconds'], d['diag']['step_ms_min_med_max'])"
timeout -k 10 300 python3 -u bench.py --config deep --steps 3 --warmup 1 > $D/deep.json 2> $D/deep.err || { echo "deep failed"; tail -30 $D/deep.err; exit 1; }
python3 -c "import json; d=json.loads(open('$D/deep.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['infer_rows_x_models_per_sec'], d['fp8_leaf_inference'])"
bash scripts/dp_rehearsal_large.sh

#!/bin/bash
# Round 3: KNN two-donor fast pass + deferred held-out imputation: tests, KNN rates, the headline.
set -o pipefail
D=gpurun_out/r3g
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_prep_gpu.py tests/test_bench_parity_gpu.py tests/test_infer_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
for k in direct fast; do
  HFENS_KNN_KERNEL=$k timeout -k 10 300 python3 scripts/probes/knn_probe.py 100000 300000 > $D/knn_$k.log 2>&1 || { echo "probe $k failed"; tail -20 $D/knn_$k.log; exit 1; }
  echo "== $k"; grep rows $D/knn_$k.log
done
HFENS_TRACE_HOST=1 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $D/headline.json 2> $D/headline.err || { echo "headline failed"; tail -30 $D/headline.err; exit 1; }
grep "^\[host\]" $D/headline.err | tail -1
python3 -c "import json; d=json.loads(open('$D/headline.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['auroc'], d['config']['stage_seconds'], d['diag']['step_ms_min_med_max'])"

#!/bin/bash
# Round 6: persistent GBC loop for the stacking batch (A/B), its tests; step-outlier probe (100 steps).
set -o pipefail
O=gpurun_out/r6m
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "persistent or device_bases or prelaunch" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
run() {  # run TAG ENV...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_$tag.json 2> $O/b_$tag.err || { echo "$tag failed"; tail -20 $O/b_$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])")"
}
tl() {
  local tag=$1; shift
  env "$@" HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 8 --warmup 3 > $O/tl_$tag.json 2> $O/tl_$tag.err || { echo "tl $tag failed"; tail -20 $O/tl_$tag.err; exit 1; }
  grep "^\[dev\]" $O/tl_$tag.err | tail -2 | head -1 | cut -c1-900
}
run base && run pst HFENS_GBDT_PERSIST_STACK=1 && run base2 && run pst2 HFENS_GBDT_PERSIST_STACK=1 && tl pst HFENS_GBDT_PERSIST_STACK=1 && timeout -k 10 300 python scripts/probes/step_outliers.py 100 > $O/outliers.log 2>&1 && tail -1 $O/outliers.log | cut -c1-1500

#!/bin/bash
# Round 5: cascade-seeded working-set SMO — the seed kernel and cascade tests, the SVC / stacking
# GPU tests, timelines with the cascade on / off, the driver's headline command.
set -o pipefail
O=gpurun_out/r5i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_svm_ws_gpu.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_ws.log 2>&1 || { echo "pytest ws failed"; tail -40 $O/pytest_ws.log; exit 1; }
tail -2 $O/pytest_ws.log
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_bench_parity_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "svc or smo or stack or bench_parity or plan_ahead or develop" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # run TAG ENV...
  local tag=$1; shift
  env "$@" HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 6 --warmup 3 > $O/tl_$tag.json 2> $O/tl_$tag.err || { echo "$tag failed"; tail -20 $O/tl_$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.loads(open('$O/tl_$tag.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['auroc'], d['diag']['step_ms_min_med_max'])")"
  grep "^\[dev\]" $O/tl_$tag.err | tail -2 | head -1 | cut -c1-300
}
run cascade HFENS_SVM_CASCADE=1
run cold HFENS_SVM_CASCADE=0
run cascade_p1000 HFENS_SVM_CASCADE=1 HFENS_SVM_CASCADE_PART=1000
run cascade_eps03 HFENS_SVM_CASCADE=1 HFENS_SVM_CASCADE_EPS=0.03
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print('bench', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"
timeout -k 10 200 python scripts/ws_stats.py > $O/ws_stats.log 2>&1 && grep -E "^q |^inner|problem" $O/ws_stats.log | head -8

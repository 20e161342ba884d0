#!/bin/bash
# Round 5: the SVC batch prelaunched under the LassoCV path — timelines (on / off), targeted GPU
# tests, the driver's headline command.
set -o pipefail
O=gpurun_out/r5d
mkdir -p $O
run() {  # run TAG ENV...
  local tag=$1; shift
  env "$@" HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 6 --warmup 3 > $O/tl_$tag.json 2> $O/tl_$tag.err || { echo "$tag failed"; tail -20 $O/tl_$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.loads(open('$O/tl_$tag.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['auroc'])")"
  grep "^\[dev\]" $O/tl_$tag.err | tail -1 | cut -c1-400
  grep "^\[host\]" $O/tl_$tag.err | tail -1 | cut -c1-900
}
run pre HFENS_PRELAUNCH_SVC=1
run nopre HFENS_PRELAUNCH_SVC=0
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_bench_parity_gpu.py tests/test_prep_gpu.py tests/test_svm_ws_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "prelaunch or stump_ranks_device or device_bases or bench_parity or device_svc_oof or plan_ahead or lasso" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print('bench', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"

#!/bin/bash
# Round 5: host-sync-free base fits with the bins copy on the aux stream — timelines, targeted
# GPU tests, the driver's headline command on both paths.
set -o pipefail
O=gpurun_out/r5c
mkdir -p $O
run() {  # run TAG ENV...
  local tag=$1; shift
  env "$@" HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 6 --warmup 3 > $O/tl_$tag.json 2> $O/tl_$tag.err || { echo "$tag failed"; tail -20 $O/tl_$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.loads(open('$O/tl_$tag.json').read().strip().splitlines()[-1]);print(d['ms_per_step'])")"
  grep "^\[dev\]" $O/tl_$tag.err | tail -1 | cut -c1-400
}
run new HFENS_DEVICE_BASES=1
run old HFENS_DEVICE_BASES=0 HFENS_BIN_AHEAD=0
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_bench_parity_gpu.py tests/test_prep_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k "stump_ranks_device or device_bases or persistent or bench_parity or knn_imputer or device_svc_oof or plan_ahead" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -30 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
HFENS_DEVICE_BASES=0 HFENS_BIN_AHEAD=0 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_old.json 2> $O/bench_old.err || { echo "bench old failed"; exit 1; }
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_new.json 2> $O/bench_new.err || { echo "bench new failed"; exit 1; }
for f in old new; do python3 -c "import json;d=json.loads(open('$O/bench_$f.json').read().strip().splitlines()[-1]);print('$f', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"; done

#!/bin/bash
# Round 6: the speculative stack finished before the LassoCV tail (host waits overlap).
set -o pipefail
O=gpurun_out/r6s
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_prep_gpu.py tests/test_svm_ws_gpu.py tests/test_train_gpu.py tests/test_bench_parity_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "lasso or ws or svc or prelaunch or speculat or early_read or device_bases or task_policy or bench_shape or cycles or persistent" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # run TAG ENV...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_$tag.json 2> $O/b_$tag.err || { echo "$tag failed"; tail -20 $O/b_$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])")"
}
tl() {
  local tag=$1; shift
  env "$@" HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 8 --warmup 3 > $O/tl_$tag.json 2> $O/tl_$tag.err || { echo "tl $tag failed"; tail -20 $O/tl_$tag.err; exit 1; }
  grep "^\[dev\]" $O/tl_$tag.err | tail -2 | head -1 | cut -c1-900
  grep "^\[host\]" $O/tl_$tag.err | tail -2 | head -1 | tr ' ' '\n' | grep -v ws_chunk | tr '\n' ' ' | cut -c1-1800; echo
}
run fbl && run nofbl HFENS_FINISH_BEFORE_LASSO=0 && run fbl2 && run nofbl2 HFENS_FINISH_BEFORE_LASSO=0 && tl fbl

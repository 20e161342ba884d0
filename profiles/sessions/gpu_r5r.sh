#!/bin/bash
# Round 5: speculative LassoCV selection (SVC batch under the CV paths) — tests, timelines, bench.
set -o pipefail
O=gpurun_out/r5r
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_train_gpu.py tests/test_bench_parity_gpu.py tests/test_prep_gpu.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider -k "speculation or prelaunch or plan_ahead or develop or bench_parity or lasso or stack" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
run() {  # run TAG ENV...
  local tag=$1; shift
  env "$@" HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 8 --warmup 3 > $O/tl_$tag.json 2> $O/tl_$tag.err || { echo "$tag failed"; tail -20 $O/tl_$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.loads(open('$O/tl_$tag.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['auroc'], d['diag']['step_ms_min_med_max'])")"
  grep "^\[dev\]" $O/tl_$tag.err | tail -2 | head -1 | cut -c1-400
  grep "^\[host\]" $O/tl_$tag.err | tail -2 | head -1 | tr ' ' '\n' | grep -v ws_chunk | tr '\n' ' ' | cut -c1-1000; echo
}
run spec HFENS_SVM_WS_AHEAD=40
run nospec HFENS_SVM_WS_AHEAD=40 HFENS_LASSO_SPECULATE=0
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print('bench', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"

#!/bin/bash
# Round 6: the whole stacking fit prelaunched on the early speculative selection (before the LassoCV
# grid read); task policy on the same path.  Targeted tests, bench, traced timeline.
set -o pipefail
O=gpurun_out/r6b
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_prep_gpu.py tests/test_bench_parity_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "prelaunch or speculat or early_read or plan_ahead or device_bases or device_svc_oof or task_policy or lasso or bench_shape" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -3 $O/pytest.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -20 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print('bench', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"
HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 8 --warmup 3 > $O/tl.json 2> $O/tl.err || { echo "tl failed"; tail -20 $O/tl.err; exit 1; }
grep "^\[dev\]" $O/tl.err | tail -2 | head -1 | cut -c1-900
grep "^\[host\]" $O/tl.err | tail -2 | head -1 | tr ' ' '\n' | grep -v ws_chunk | tr '\n' ' ' | cut -c1-1800; echo

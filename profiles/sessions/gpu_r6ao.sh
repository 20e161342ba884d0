#!/bin/bash
# Round 6: batched scaler attributes, lazy OOF items, one test-fold upload (int8 radix sort), one-compare fold masks.
set -o pipefail
O=gpurun_out/r6ao
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_svm_ws_gpu.py tests/test_train_gpu.py tests/test_bench_parity_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "ws or svc or platt or prelaunch or speculat or device_bases or device_svc_oof or merged_oof or task_policy or bench_shape or plan_ahead" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 300 python -u scripts/probes/preparts_profile.py > $O/preparts.log 2>&1 || { echo "preparts failed"; tail -30 $O/preparts.log; exit 1; }
grep "window wall" $O/preparts.log
for t in B1 B2 B3; do
  if [ ${t:0:1} = A ]; then export HFENS_PLAN_JOIN_LATE=0; else export HFENS_PLAN_JOIN_LATE=1; fi
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_$t.json 2> $O/b_$t.err || { echo "bench failed"; tail -20 $O/b_$t.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b_$t.json').read().strip().splitlines()[-1]);print('bench $t', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'], d['diag']['svm']['ws_rounds_max'], d['diag']['svm']['ws_pairs_max'])"; done
unset HFENS_PLAN_JOIN_LATE
HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 8 --warmup 3 > $O/tl.json 2> $O/tl.err || { echo "tl failed"; tail -20 $O/tl.err; exit 1; }
grep "^\[dev\]" $O/tl.err | tail -2 | head -1 | cut -c1-900
grep "^\[host\]" $O/tl.err | tail -2 | head -1 | tr " " "\n" | grep -v ws_chunk | tr "\n" " " | cut -c1-1200; echo

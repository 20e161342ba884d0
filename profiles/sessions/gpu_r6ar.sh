#!/bin/bash
# Round 6: the fit's early read-backs polled on their pinned data (utils.hostread: selection, early SMO
# read, Platt pairs, γ, LR and base-model guards)
# instead of waiting on their events: SVC / stacking tests, traced medians, bench x3.
set -o pipefail
O=gpurun_out/r6ar
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_svm_ws_gpu.py tests/test_train_gpu.py tests/test_bench_parity_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "ws or svc or platt or prelaunch or speculat or device_bases or device_svc_oof or merged_oof or task_policy or bench_shape or plan_ahead" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 12 --warmup 3 > $O/tl.json 2> $O/tl.err || { echo "tl failed"; tail -20 $O/tl.err; exit 1; }
python3 scripts/probes/tl_summary.py $O/tl.err 3
grep "^\[host\]" $O/tl.err | tail -2 | head -1 | tr " " "\n" | grep -E "^(develop|lasso_best_read|selected|cols_synced|finish_in|svc_early_wait|svc_early_synced|svc_host_read|svc_platt_read|svc_finished)=" | tr "\n" " "; echo
grep "^\[dev\]" $O/tl.err | tail -2 | head -1 | cut -c1-400
for t in 1 2 3 4; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_$t.json 2> $O/b_$t.err || { echo "bench failed"; tail -20 $O/b_$t.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b_$t.json').read().strip().splitlines()[-1]);print('bench $t', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'], d['diag']['svm']['ws_pairs_max'])"; done

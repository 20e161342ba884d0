#!/bin/bash
# Round 6: the Platt fits over 8 workgroups per fit (platt_coop_kernel): SVC / Platt / OOF tests,
# traced tail medians (decision time), bench x2.
set -o pipefail
O=gpurun_out/r6bl
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_svm_ws_gpu.py tests/test_train_gpu.py tests/test_bench_parity_gpu.py tests/test_svc_scale_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "ws or svc or platt or prelaunch or speculat or task_policy or bench_shape or resolve or oof or decision" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 12 --warmup 3 > $O/tl.json 2> $O/tl.err || { echo "tl failed"; tail -20 $O/tl.err; exit 1; }
python3 scripts/probes/tl_summary.py $O/tl.err 3 | head -3
for t in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_$t.json 2> $O/b_$t.err || { echo "bench failed"; tail -20 $O/b_$t.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b_$t.json').read().strip().splitlines()[-1]);print('bench $t', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'], d['diag']['svm'].get('ws_critical'))"; done

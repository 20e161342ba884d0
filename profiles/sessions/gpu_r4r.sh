#!/bin/bash
# round 4: fold-SVC bookkeeping overlapped with the meta fit — device OOF test, headline bench
# with and without it (alternating, two each), host/device timeline
set -o pipefail
D=gpurun_out/r4r
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_train_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "device_svc_oof or stacking" > $D/pytest_oof.log 2>&1 || { echo "pytest failed"; tail -40 $D/pytest_oof.log; exit 1; }
tail -2 $D/pytest_oof.log
run() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $D/$name.json 2> $D/$name.err || { echo "$name failed"; tail -30 $D/$name.err; return 1; }
  python -c "import json; d=json.loads(open('$D/$name.json').read().strip().split('\n')[-1]); print('$name', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"
}
run defer1 HFENS_X=0 &&
run nodefer1 HFENS_DEFER_FOLD_SVC=0 &&
run defer2 HFENS_X=0 &&
run nodefer2 HFENS_DEFER_FOLD_SVC=0 &&
HFENS_TRACE_HOST=1 timeout -k 10 200 python -u scripts/probes/ws_events.py > $D/ev_host.log 2>&1 || { echo "events failed"; tail -30 $D/ev_host.log; exit 1; }
tail -25 $D/ev_host.log

#!/bin/bash
# Round 6: host tail trims (SVC set_fitted before the Platt read, base guards resolved early, meta LR
# models set at launch): stacking / SVC / LR tests, then on vs off traced medians interleaved, bench x2.
set -o pipefail
O=gpurun_out/r6bp
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_svm_ws_gpu.py tests/test_train_gpu.py tests/test_bench_parity_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in a b; do for v in 1 0; do
  HFENS_META_PRESET=$v HFENS_BASES_EARLY_RESOLVE=$v HFENS_SVC_SET_BEFORE_PLATT=$v HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 12 --warmup 3 > $O/tl_${v}$r.json 2> $O/tl_${v}$r.err || { echo "tl failed"; tail -20 $O/tl_${v}$r.err; exit 1; }
  echo "trims=$v ($r)"; { python3 scripts/probes/tl_summary.py $O/tl_${v}$r.err 3; python3 scripts/probes/tail_host.py $O/tl_${v}$r.err 3; } | tee $O/tl_${v}${r}_medians.log
done; done
for t in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_$t.json 2> $O/b_$t.err || { echo "bench failed"; tail -20 $O/b_$t.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b_$t.json').read().strip().splitlines()[-1]);print('bench $t', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"; done

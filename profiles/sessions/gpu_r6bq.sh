#!/bin/bash
# Round 6: host_store read-backs (kernel system-scope stores into pinned memory instead of an async
# copy): stage/landed tests, latency probe, stacking tests, traced on/off medians interleaved, bench x2.
set -o pipefail
O=gpurun_out/r6bq
mkdir -p $O
timeout -k 10 200 python -u -m pytest tests/test_hostread.py -x -v --timeout 100 --timeout-method thread -p no:cacheprovider > $O/pytest_hr.log 2>&1 || { echo "pytest hostread failed"; tail -60 $O/pytest_hr.log; exit 1; }
tail -2 $O/pytest_hr.log
timeout -k 10 120 python scripts/probes/hostread_latency.py 200 2>&1 | tee $O/latency.log
timeout -k 10 700 python -u -m pytest tests/test_svm_ws_gpu.py tests/test_train_gpu.py tests/test_bench_parity_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in a b; do for v in 1 0 t; do
  k=$v; t=1; if [ $v = t ]; then k=1; t=0; fi
  HFENS_META_PRESET=$t HFENS_BASES_EARLY_RESOLVE=$t HFENS_SVC_SET_BEFORE_PLATT=$t HFENS_HOSTREAD_KERNEL=$k HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 12 --warmup 3 > $O/tl_${v}$r.json 2> $O/tl_${v}$r.err || { echo "tl failed"; tail -20 $O/tl_${v}$r.err; exit 1; }
  echo "kernel=$k trims=$t ($r)"; { python3 scripts/probes/tl_summary.py $O/tl_${v}$r.err 3; python3 scripts/probes/tail_host.py $O/tl_${v}$r.err 3; } | tee $O/tl_${v}${r}_medians.log
done; done
for t in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_$t.json 2> $O/b_$t.err || { echo "bench failed"; tail -20 $O/b_$t.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b_$t.json').read().strip().splitlines()[-1]);print('bench $t', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"; done

#!/bin/bash
# Round 6: meta LR launch gap (guards computed behind the solve, cached penalty mask): LR / stacking
# tests, traced medians x2 (oof→lr_kernel was 0.27–0.29 ms in r6bn/r6bp/r6bq), bench x1.
set -o pipefail
O=gpurun_out/r6bu
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests/test_train_gpu.py tests/test_bench_parity_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for r in a b; do
  HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 12 --warmup 3 > $O/tl_$r.json 2> $O/tl_$r.err || { echo "tl failed"; tail -20 $O/tl_$r.err; exit 1; }
  python3 scripts/probes/tl_summary.py $O/tl_$r.err 3 | tee $O/tl_${r}_medians.log
done
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_1.json 2> $O/b_1.err || { echo "bench failed"; tail -20 $O/b_1.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/b_1.json').read().strip().splitlines()[-1]);print('bench', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"

#!/bin/bash
# round 4: held-out KNN after the LassoCV path — timeline + bench ×2 + the prep/train tests
set -o pipefail
D=gpurun_out/r4aa
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_prep_gpu.py tests/test_robustness.py tests/test_bench_parity_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 4 --warmup 2 > $D/trace.json 2> $D/trace.err || { echo "trace failed"; tail -30 $D/trace.err; exit 1; }
grep -E "^\[(dev|host)\]" $D/trace.err | tail -2
for k in 1 2; do
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $D/bench$k.json 2> $D/bench$k.err || { echo "bench failed"; tail -30 $D/bench$k.err; exit 1; }
  python -c "import json; d=json.loads(open('$D/bench$k.json').read().strip().split('\n')[-1]); print('bench$k', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"
done

#!/bin/bash
# Round 5: post-SMO chain beside the largest (final-only) solver group — tests, timelines, bench A/B.
set -o pipefail
O=gpurun_out/r5az
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_svm_ws_gpu.py tests/test_bench_parity_gpu.py tests/test_train_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  for m in 1 0; do
    HFENS_SVM_LATE_GROUP=$m HFENS_TRACE_DEV=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_${m}_$i.json 2> $O/bench_${m}_$i.err || { echo "bench failed"; tail -20 $O/bench_${m}_$i.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/bench_${m}_$i.json').read().strip().splitlines()[-1]);print('late=$m', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"
    grep "^\[dev\]" $O/bench_${m}_$i.err | tail -2 | head -1 | cut -c1-500
  done
done

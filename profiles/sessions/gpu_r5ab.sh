#!/bin/bash
# Round 5: host trims (no column maps on the ws path, 48 seeded rounds ahead) — tests, timeline, bench.
set -o pipefail
O=gpurun_out/r5ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_svm_ws_gpu.py tests/test_train_gpu.py tests/test_bench_parity_gpu.py tests/test_prep_gpu.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider -k "ws or svc or stack or develop or speculation or bench_parity or lasso or prep" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 8 --warmup 3 > $O/tl.json 2> $O/tl.err || { echo "tl failed"; tail -20 $O/tl.err; exit 1; }
grep "^\[dev\]" $O/tl.err | tail -2 | head -1 | cut -c1-400
grep "^\[host\]" $O/tl.err | tail -2 | head -1 | tr ' ' '\n' | grep -v ws_chunk | tr '\n' ' ' | cut -c1-900; echo
for i in 1 2; do
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench$i.json 2> $O/bench$i.err || { echo "bench failed"; tail -5 $O/bench$i.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench$i.json').read().strip().splitlines()[-1]);print('bench', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"
done

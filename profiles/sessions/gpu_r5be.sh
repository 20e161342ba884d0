#!/bin/bash
# Round 5: split-K cascade seed gradient — tests, headline bench, seed kernel time.
set -o pipefail
O=gpurun_out/r5be
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_svm_ws_gpu.py tests/test_bench_parity_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for i in 1 2; do
  HFENS_TRACE_DEV=1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_$i.json 2> $O/bench_$i.err || { echo "bench failed"; tail -20 $O/bench_$i.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_$i.json').read().strip().splitlines()[-1]);print('bench', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"
  grep "^\[dev\]" $O/bench_$i.err | tail -2 | head -1 | cut -c1-300
done
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 3 --warmup 1 > $O/prof.json 2> $O/prof.err || { echo "prof failed"; tail -20 $O/prof.err; exit 1; }
grep -E "ws_seed" $O/prof/run_kernel_stats.csv | cut -c1-200
rm -f $O/prof/run_kernel_trace.csv

#!/bin/bash
# Round 5: device-built cascade parts (one group) — ws tests, timelines, bench.
set -o pipefail
O=gpurun_out/r5o
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_svm_ws_gpu.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_ws.log 2>&1 || { echo "pytest ws failed"; tail -40 $O/pytest_ws.log; exit 1; }
tail -2 $O/pytest_ws.log
run() {  # run TAG ENV...
  local tag=$1; shift
  env "$@" HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 8 --warmup 3 > $O/tl_$tag.json 2> $O/tl_$tag.err || { echo "$tag failed"; tail -20 $O/tl_$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.loads(open('$O/tl_$tag.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['auroc'], d['diag']['step_ms_min_med_max'])")"
  grep "^\[dev\]" $O/tl_$tag.err | tail -2 | head -1 | cut -c1-400
  grep "^\[host\]" $O/tl_$tag.err | tail -2 | head -1 | tr ' ' '\n' | grep -v ws_chunk | tr '\n' ' ' | cut -c1-1000; echo
}
run base
run graph HFENS_SVM_WS_GRAPH=all
run graph_r6 HFENS_SVM_WS_GRAPH=all HFENS_SVM_CASCADE_ROUNDS=6
run graph_p1250 HFENS_SVM_WS_GRAPH=all HFENS_SVM_CASCADE_PART=1250
run graph_q512 HFENS_SVM_WS_GRAPH=all HFENS_SVM_WS_Q=512
run graph_q512_f3 HFENS_SVM_WS_GRAPH=all HFENS_SVM_WS_Q=512 HFENS_SVM_WS_FRAC=0.3
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print('bench', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"
HFENS_SVM_WS_GRAPH=all timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_graph.json 2> $O/bench_graph.err || { echo "bench failed"; tail -5 $O/bench_graph.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench_graph.json').read().strip().splitlines()[-1]);print('bench_graph', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"

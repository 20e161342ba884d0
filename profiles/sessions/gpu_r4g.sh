#!/bin/bash
# round 4: host-enqueue variants of the q = 1024 working-set rounds on the headline
set -o pipefail
D=gpurun_out/r4g
mkdir -p $D
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $D/$name.json 2> $D/$name.err || { echo "$name failed"; tail -30 $D/$name.err; return 1; }
  python -c "import json; d=json.loads(open('$D/$name.json').read().strip().split('\n')[-1]); print('$name', d['ms_per_step'], d['diag']['step_ms_min_med_max'])"
}
run base HFENS_X=0 &&
run graph_all HFENS_SVM_WS_GRAPH=all &&
run enq16 HFENS_SVM_WS_ENQ_CHUNK=16 &&
run ahead40 HFENS_SVM_WS_AHEAD=40 &&
run graph_all_16x3 HFENS_SVM_WS_GRAPH=all HFENS_SVM_WS_GRAPH_CHUNK=16 HFENS_SVM_WS_AHEAD=48 &&
run base2 HFENS_X=0

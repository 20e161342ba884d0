#!/bin/bash
# Round 5: cascade with graph-replayed rounds / fewer rounds ahead — host+device timelines.
set -o pipefail
O=gpurun_out/r5k
mkdir -p $O
run() {  # run TAG ENV...
  local tag=$1; shift
  env "$@" HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 8 --warmup 3 > $O/tl_$tag.json 2> $O/tl_$tag.err || { echo "$tag failed"; tail -20 $O/tl_$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.loads(open('$O/tl_$tag.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['auroc'], d['diag']['step_ms_min_med_max'])")"
  grep "^\[dev\]" $O/tl_$tag.err | tail -2 | head -1 | cut -c1-400
  grep "^\[host\]" $O/tl_$tag.err | tail -2 | head -1 | tr ' ' '\n' | grep -v ws_chunk | tr '\n' ' ' | cut -c1-900; echo
}
run base HFENS_SVM_CASCADE_ROUNDS=8 HFENS_SVM_CASCADE_PART=1600
run graph HFENS_SVM_CASCADE_ROUNDS=8 HFENS_SVM_CASCADE_PART=1600 HFENS_SVM_WS_GRAPH=all
run ahead40 HFENS_SVM_CASCADE_ROUNDS=8 HFENS_SVM_CASCADE_PART=1600 HFENS_SVM_WS_AHEAD=40
run graph_ahead40 HFENS_SVM_CASCADE_ROUNDS=8 HFENS_SVM_CASCADE_PART=1600 HFENS_SVM_WS_GRAPH=all HFENS_SVM_WS_AHEAD=40
run graph_p2000 HFENS_SVM_CASCADE_ROUNDS=8 HFENS_SVM_CASCADE_PART=2000 HFENS_SVM_WS_GRAPH=all

#!/bin/bash
# Round 5: after removing the host-blocking uploads (fold masks, meta LR penalty, GBDT bin edges).
set -o pipefail
O=gpurun_out/r5n
mkdir -p $O
run() {  # run TAG ENV...
  local tag=$1; shift
  env "$@" HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 8 --warmup 3 > $O/tl_$tag.json 2> $O/tl_$tag.err || { echo "$tag failed"; tail -20 $O/tl_$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.loads(open('$O/tl_$tag.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['auroc'], d['diag']['step_ms_min_med_max'])")"
  grep "^\[dev\]" $O/tl_$tag.err | tail -2 | head -1 | cut -c1-400
  grep "^\[host\]" $O/tl_$tag.err | tail -2 | head -1 | tr ' ' '\n' | grep -v ws_chunk | tr '\n' ' ' | cut -c1-1400; echo
}
run base
run graph HFENS_SVM_WS_GRAPH=all
run p2000 HFENS_SVM_CASCADE_PART=2000
run cold HFENS_SVM_CASCADE=0
timeout -k 10 300 python scripts/probes/sync_debug.py > $O/sync.log 2>&1 && grep -v amdgpu.ids $O/sync.log | cut -c100-330 | tail -30
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print('bench', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"

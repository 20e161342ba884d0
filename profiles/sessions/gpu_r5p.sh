#!/bin/bash
# Round 5: per-group round timeline of the seeded working-set solve; rounds-ahead variants.
set -o pipefail
O=gpurun_out/r5p
mkdir -p $O
timeout -k 10 200 python scripts/probes/ws_events.py > $O/ws_events.log 2>&1 || { echo "events failed"; tail -20 $O/ws_events.log; exit 1; }
grep -v amdgpu.ids $O/ws_events.log | tail -12 | cut -c1-700
run() {  # run TAG ENV...
  local tag=$1; shift
  env "$@" HFENS_TRACE_DEV=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/tl_$tag.json 2> $O/tl_$tag.err || { echo "$tag failed"; tail -20 $O/tl_$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.loads(open('$O/tl_$tag.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['auroc'], d['diag']['step_ms_min_med_max'])")"
  grep "^\[dev\]" $O/tl_$tag.err | tail -2 | head -1 | cut -c1-300
}
run base
run ahead40 HFENS_SVM_WS_AHEAD=40
run base2
run ahead32 HFENS_SVM_WS_AHEAD=32

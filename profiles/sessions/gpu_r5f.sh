#!/bin/bash
# Round 5: why the prelaunched SVC batch runs slower — switch matrix with device timelines and
# per-group SMO events.
set -o pipefail
O=gpurun_out/r5f
mkdir -p $O
run() {  # run TAG ENV...
  local tag=$1; shift
  env "$@" HFENS_TRACE_DEV=1 timeout -k 10 200 python bench.py --steps 6 --warmup 3 > $O/tl_$tag.json 2> $O/tl_$tag.err || { echo "$tag failed"; tail -20 $O/tl_$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.loads(open('$O/tl_$tag.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['auroc'], d['diag']['step_ms_min_med_max'])")"
  grep "^\[dev\]" $O/tl_$tag.err | tail -2 | head -1 | cut -c1-300
}
run pre_init HFENS_PRELAUNCH_SVC=1
run nopre_init HFENS_PRELAUNCH_SVC=0
run pre_noinit HFENS_PRELAUNCH_SVC=1 HFENS_INIT_STREAMS=0
run pre_noearly HFENS_PRELAUNCH_SVC=1 HFENS_EARLY_META=0
run pre_nobases HFENS_PRELAUNCH_SVC=1 HFENS_DEVICE_BASES=0
HFENS_WS_EVENTS=1 timeout -k 10 200 python scripts/probes/ws_events.py > $O/ws_events_pre.log 2>&1 || echo "ws_events failed"
HFENS_PRELAUNCH_SVC=0 HFENS_WS_EVENTS=1 timeout -k 10 200 python scripts/probes/ws_events.py > $O/ws_events_nopre.log 2>&1 || echo "ws_events nopre failed"
tail -8 $O/ws_events_pre.log; tail -8 $O/ws_events_nopre.log

#!/bin/bash
# Round 5: hardware-queue hypothesis for the prelaunched SVC batch's slow SMO group —
# GPU_MAX_HW_QUEUES 4 (box default) vs 8 / 16, prelaunch on/off, early meta on/off.
set -o pipefail
O=gpurun_out/r5g
mkdir -p $O
run() {  # run TAG ENV...
  local tag=$1; shift
  env "$@" HFENS_TRACE_DEV=1 timeout -k 10 200 python bench.py --steps 6 --warmup 3 > $O/tl_$tag.json 2> $O/tl_$tag.err || { echo "$tag failed"; tail -20 $O/tl_$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.loads(open('$O/tl_$tag.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['auroc'], d['diag']['step_ms_min_med_max'])")"
  grep "^\[dev\]" $O/tl_$tag.err | tail -2 | head -1 | cut -c1-200
}
run q4_pre GPU_MAX_HW_QUEUES=4 HFENS_PRELAUNCH_SVC=1
run q8_pre GPU_MAX_HW_QUEUES=8 HFENS_PRELAUNCH_SVC=1
run q16_pre GPU_MAX_HW_QUEUES=16 HFENS_PRELAUNCH_SVC=1
run q8_pre_noearly GPU_MAX_HW_QUEUES=8 HFENS_PRELAUNCH_SVC=1 HFENS_EARLY_META=0
run q8_nopre GPU_MAX_HW_QUEUES=8 HFENS_PRELAUNCH_SVC=0
run q16_nopre GPU_MAX_HW_QUEUES=16 HFENS_PRELAUNCH_SVC=0
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
HFENS_PRELAUNCH_SVC=1 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt_pre -o kt -- python3 bench.py --steps 1 --warmup 1 > $O/kt_pre.log 2>&1 || { echo "kt pre failed"; tail -5 $O/kt_pre.log; exit 1; }
HFENS_PRELAUNCH_SVC=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt_nopre -o kt -- python3 bench.py --steps 1 --warmup 1 > $O/kt_nopre.log 2>&1 || { echo "kt nopre failed"; tail -5 $O/kt_nopre.log; exit 1; }
echo ok

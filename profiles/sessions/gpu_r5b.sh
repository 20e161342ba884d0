#!/bin/bash
# Round 5: A/B of the host-sync-free base fits — which piece slows the SMO (device timelines).
set -o pipefail
O=gpurun_out/r5b
mkdir -p $O
run() {  # run TAG ENV...
  local tag=$1; shift
  env "$@" HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 6 --warmup 3 > $O/tl_$tag.json 2> $O/tl_$tag.err || { echo "$tag failed"; tail -20 $O/tl_$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.loads(open('$O/tl_$tag.json').read().strip().splitlines()[-1]);print(d['ms_per_step'])")"
  grep "^\[dev\]" $O/tl_$tag.err | tail -1 | cut -c1-400
}
run new HFENS_DEVICE_BASES=1
run old HFENS_DEVICE_BASES=0 HFENS_BIN_AHEAD=0
run nobins HFENS_DEVICE_BASES=1 HFENS_BIN_AHEAD=0
run noearly HFENS_DEVICE_BASES=1 HFENS_EARLY_META=0
run old_noearly HFENS_DEVICE_BASES=0 HFENS_BIN_AHEAD=0 HFENS_EARLY_META=0
run new2 HFENS_DEVICE_BASES=1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt_new -o kt -- python3 bench.py --steps 2 --warmup 1 > $O/kt_new.log 2>&1 || { echo "kt new failed"; tail -5 $O/kt_new.log; exit 1; }
HFENS_DEVICE_BASES=0 HFENS_BIN_AHEAD=0 timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $O/kt_old -o kt -- python3 bench.py --steps 2 --warmup 1 > $O/kt_old.log 2>&1 || { echo "kt old failed"; tail -5 $O/kt_old.log; exit 1; }
find $O -name "*kernel_trace.csv" | head

#!/bin/bash
# Driver-vs-builder gap diagnosis: the exact driver command, then the same with
# one knob changed at a time, then under host CPU contention.  Every GPU step has its own limit;
# stop at the first failure.
set -o pipefail
mkdir -p gpurun_out/diag
D=gpurun_out/diag
{ echo "nproc=$(nproc)"; cat /proc/loadavg; echo "affinity=$(python3 -c 'import os;print(len(os.sched_getaffinity(0)))')"; } > $D/host.txt
run() {  # run TAG ENV...
  local tag=$1; shift
  timeout -k 10 240 env "$@" python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/$tag.json 2> $D/$tag.err \
    || { echo "$tag failed"; tail -20 $D/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/$tag.json')); print('$tag', d['ms_per_step'], d['config']['stage_seconds'], d['diag']['host_cpu_fraction'], d['diag']['step_ms_min_med_max'])"
}
run driver HFENS_X=0
run trace HFENS_TRACE_HOST=1
run nocoop HFENS_SMO_COOP=0
run serial HFENS_CONCURRENT_BASES=0
# host contention: 16 busy loops (bounded by their own timeout) beside the bench
pids=""
for i in $(seq 16); do timeout 200 sh -c 'while :; do :; done' & pids="$pids $!"; done
run contended HFENS_X=0
kill $pids 2>/dev/null
wait 2>/dev/null
true

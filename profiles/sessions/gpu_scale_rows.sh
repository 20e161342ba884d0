#!/bin/bash
# Full-ensemble development fit at growing row counts (BASELINE config 3 path, one GPU):
# per-stage medians and the SVC solver that ran.  Each step has its own limit; stop at the first
# failure.
set -o pipefail
D=gpurun_out/rows
mkdir -p $D
run() {  # run TAG SECONDS ARGS...
  local tag=$1 secs=$2; shift 2
  timeout -k 10 $secs python3 -u bench.py "$@" > $D/$tag.json 2> $D/$tag.err || { echo "$tag failed"; tail -30 $D/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/$tag.json')); print('$tag', d['ms_per_step'], d['value'], d['auroc'], d['config']['stage_seconds'], d['diag']['svm'])"
}
[ -z "$ONLY1M" ] && run r30k 200 --rows 30000 --steps 1 --warmup 1
[ -z "$ONLY1M" ] && run r100k 300 --rows 100000 --steps 1 --warmup 1
run r1m 900 --rows 1000000 --steps 1 --warmup 0

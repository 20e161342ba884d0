#!/bin/bash
# Performance pass: headline bench, GBDT-only 1M (cfg 3 analog), deep ensemble (cfg 5), and a
# kernel-trace profile of the headline.  Each GPU step has its own limit; stop at the first failure.
set -o pipefail
D=gpurun_out/perf
mkdir -p $D
run() {  # run TAG SECONDS ARGS...
  local tag=$1 secs=$2; shift 2
  timeout -k 10 $secs python3 -u bench.py "$@" > $D/$tag.json 2> $D/$tag.err || { echo "$tag failed"; tail -30 $D/$tag.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/$tag.json')); print('$tag', d['ms_per_step'], d['value'], d.get('auroc'), d['config'].get('stage_seconds'), (d.get('diag') or {}).get('gbdt_path'))"
}
run headline 300 --gpus 1 --steps 20 --warmup 5
run gbdt1m 300 --config gbdt --steps 5 --warmup 1
run deep 400 --config deep --steps 2 --warmup 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o bench --output-format csv -- python3 bench.py --steps 3 --warmup 2 > $D/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $D/prof.log; exit 1; }
find $D/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $D/headline_kernel_stats.csv
head -16 $D/headline_kernel_stats.csv | cut -c1-200

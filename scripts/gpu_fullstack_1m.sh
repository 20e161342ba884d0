#!/bin/bash
# BASELINE config 3: the full development fit at 1M rows on one GPU (one timed step).
set -o pipefail
D=gpurun_out/fs1m
mkdir -p $D
timeout -k 10 600 python3 -u bench.py --rows 1000000 --steps 1 --warmup 0 > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -30 $D/bench.err; exit 1; }
python3 -c "import json; d=json.loads(open('$D/bench.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['auroc'], d['config']['stage_seconds'], d['diag'].get('svm'))"

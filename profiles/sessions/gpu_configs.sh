#!/bin/bash
# BASELINE configs 3 (GBC 1M), 4 (100M-row inference) and 5 (deep ensemble, fp8 leaves) on one GPU.
set -o pipefail
D=gpurun_out/configs
mkdir -p $D
run() {  # run TAG SECONDS ARGS...
  local tag=$1 secs=$2; shift 2
  timeout -k 10 $secs python3 -u bench.py "$@" > $D/$tag.json 2> $D/$tag.err || { echo "$tag failed"; tail -30 $D/$tag.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$D/$tag.json').read().strip().splitlines()[-1]); print('$tag', d['ms_per_step'], d['value'], d.get('auroc'), d.get('vs_baseline'), d.get('fp8_leaf_inference', {}) and d['fp8_leaf_inference'].get('auroc_delta'))"
}
run infer 400 --config infer --steps 10 --warmup 2
run gbdt 300 --config gbdt --steps 10 --warmup 2
run deep 400 --config deep --steps 3 --warmup 1 --subsample 0.8

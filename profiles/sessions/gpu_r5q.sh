#!/bin/bash
# Round 5: seeded working-set solve knobs — inner stop fraction, 512-thread inner solver.
set -o pipefail
O=gpurun_out/r5q
mkdir -p $O
run() {  # run TAG ENV...
  local tag=$1; shift
  env "$@" HFENS_TRACE_DEV=1 timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $O/tl_$tag.json 2> $O/tl_$tag.err || { echo "$tag failed"; tail -20 $O/tl_$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.loads(open('$O/tl_$tag.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['auroc'], d['diag']['step_ms_min_med_max'])")"
  grep "^\[dev\]" $O/tl_$tag.err | tail -2 | head -1 | cut -c1-160
}
export HFENS_SVM_WS_AHEAD=40
run base
run th512 HFENS_SVM_WS_THREADS=512
run f03 HFENS_SVM_WS_FRAC=0.3
run f01 HFENS_SVM_WS_FRAC=0.1
run f04 HFENS_SVM_WS_FRAC=0.4
run base2

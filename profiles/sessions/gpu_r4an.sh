#!/bin/bash
# round 4: A/B of the early SVC read-back on one box (alternating, 3 runs each)
set -o pipefail
D=gpurun_out/r4an
mkdir -p $D
run() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $D/$name.json 2> $D/$name.err || { echo "$name failed"; tail -30 $D/$name.err; return 1; }
  python -c "import json; d=json.loads(open('$D/$name.json').read().strip().split('\n')[-1]); print('$name', d['ms_per_step'], d['diag']['step_ms_min_med_max'])"
}
run early1 HFENS_X=0 && run late1 HFENS_SVC_EARLY_READ=0 && run early2 HFENS_X=0 && run late2 HFENS_SVC_EARLY_READ=0 && run early3 HFENS_X=0 && run late3 HFENS_SVC_EARLY_READ=0

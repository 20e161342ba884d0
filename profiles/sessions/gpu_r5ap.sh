#!/bin/bash
# Round 5: config-3 knobs — concurrent Platt-CV solves per fit, Gondzio correctors.
set -o pipefail
O=gpurun_out/r5ap
mkdir -p $O
for cfg in "3 2" "5 2" "3 1" "5 1"; do
  set -- $cfg
  HFENS_IPM_THREADS=$1 HFENS_IPM_CORRECTORS=$2 timeout -k 10 600 python -u bench.py --rows 1000000 --steps 1 --warmup 1 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { echo "bench failed"; tail -20 $O/b_$1_$2.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b_$1_$2.json').read().strip().splitlines()[-1]);print('threads $1 correctors $2:', d['ms_per_step'], d['auroc'], d['config'].get('stage_seconds'), d['diag']['svm'].get('lowrank',{}).get('ipm_iters'))"
done

#!/bin/bash
# Round 5: config-3 knobs under five IPM threads — one-workgroup Cholesky, three Gondzio correctors.
set -o pipefail
O=gpurun_out/r5bc
mkdir -p $O
for cfg in "1 2" "0 2" "1 3"; do
  set -- $cfg
  HFENS_CHOL_MW=$1 HFENS_IPM_CORRECTORS=$2 timeout -k 10 600 python -u bench.py --rows 1000000 --steps 1 --warmup 1 > $O/b_$1_$2.json 2> $O/b_$1_$2.err || { echo "bench failed"; tail -20 $O/b_$1_$2.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b_$1_$2.json').read().strip().splitlines()[-1]);print('chol_mw $1 correctors $2:', d['ms_per_step'], d['auroc'], d['config'].get('stage_seconds'), d['diag']['svm'].get('lowrank',{}).get('ipm_iters'))"
done

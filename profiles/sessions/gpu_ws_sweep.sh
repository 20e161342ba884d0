#!/bin/bash
# A/B of working-set SMO knobs on the headline (10 steps each): inner stop fraction, inner threads.
# CONFIGS="frac threads;..." overrides the list.
set -o pipefail
D=gpurun_out/wssweep
mkdir -p $D
IFS=';' read -ra CFGS <<< "${CONFIGS:-0.1 256;0.05 256;0.2 256;0.3 256;0.1 512}"
for cfg in "${CFGS[@]}"; do
  set -- $cfg
  HFENS_SVM_WS_FRAC=$1 HFENS_SVM_WS_THREADS=$2 timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $D/f$1_t$2.json 2> $D/f$1_t$2.err || { echo "run $cfg failed"; tail -20 $D/f$1_t$2.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$D/f$1_t$2.json').read().strip().splitlines()[-1]); print('frac $1 threads $2:', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['diag']['svm'].get('ws_rounds_max'), d['diag']['svm'].get('ws_pairs_max'), d['auroc'])"
done

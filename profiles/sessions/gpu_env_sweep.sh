#!/bin/bash
# A/B of environment knobs on the headline (10 steps each).  CONFIGS="A=1 B=2;A=3;..." (';' between runs).
set -o pipefail
D=gpurun_out/envsweep
mkdir -p $D
IFS=';' read -ra CFGS <<< "${CONFIGS:?set CONFIGS}"
i=0
for cfg in "${CFGS[@]}"; do
  i=$((i + 1))
  env $cfg timeout -k 10 200 python bench.py --steps 10 --warmup 3 > $D/run$i.json 2> $D/run$i.err || { echo "run [$cfg] failed"; tail -20 $D/run$i.err; exit 1; }
  python3 -c "import json; d=json.loads(open('$D/run$i.json').read().strip().splitlines()[-1]); print('[$cfg]', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['diag']['svm'].get('ws_rounds_max'), d['diag']['svm'].get('ws_pairs_max'), d['auroc'])"
done

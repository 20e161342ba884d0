#!/bin/bash
# Cooperative-SMO member-count sweep on the driver's bench command (prefetch on).
set -o pipefail
D=gpurun_out/sweep
mkdir -p $D
for w in ${WS:-2 3 4 6 8 4}; do export HFENS_SMO_COOP_RESERVE=${RES:-80}
  HFENS_SMO_COOP_MAXW=$w timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/w$w.json 2> $D/w$w.err \
    || { echo "bench failed"; tail -30 $D/w$w.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/w$w.json')); print('W=$w', d['ms_per_step'], d['config']['stage_seconds']['fit_bases(svc || gbc+lr)'], d['diag']['step_ms_min_med_max'], d['diag']['svm'])"
done

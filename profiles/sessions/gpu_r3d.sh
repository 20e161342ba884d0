#!/bin/bash
# Round 3: the fast KNN pass (same donors + rates), the driver's headline command with host marks,
# then the multi-rank rehearsals on one card.
set -o pipefail
bash scripts/probes/gpu_knn_fast.sh || exit 1
D=gpurun_out/r3d
mkdir -p $D
HFENS_TRACE_HOST=1 timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $D/headline.json 2> $D/headline.err || { echo "headline failed"; tail -30 $D/headline.err; exit 1; }
grep "^\[host\]" $D/headline.err | tail -1
python3 -c "import json; d=json.loads(open('$D/headline.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['auroc'], d['config']['stage_seconds'], d['diag']['step_ms_min_med_max'])"
RANKS="2 4" bash scripts/dp_rehearsal.sh || exit 1
bash scripts/dp_rehearsal_large.sh

#!/bin/bash
# Round 5: config-3 (1M rows) re-measure after the low-rank prelaunch fix and the matrix-core KNN filter.
set -o pipefail
O=gpurun_out/r5af
mkdir -p $O
timeout -k 10 900 python -u bench.py --rows 1000000 --steps 2 --warmup 1 > $O/fullstack_1m.json 2> $O/fullstack_1m.err || { echo "1m failed"; tail -20 $O/fullstack_1m.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/fullstack_1m.json').read().strip().splitlines()[-1]);print('1M', d['ms_per_step'], d['auroc'], d['diag'].get('step_ms_min_med_max'), d['config'].get('stage_seconds'))"
HFENS_KNN_MFMA=0 timeout -k 10 900 python -u bench.py --rows 1000000 --steps 1 --warmup 1 > $O/fullstack_1m_fma.json 2> $O/fullstack_1m_fma.err || { echo "1m fma failed"; tail -20 $O/fullstack_1m_fma.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/fullstack_1m_fma.json').read().strip().splitlines()[-1]);print('1M fma', d['ms_per_step'], d['auroc'], d['config'].get('stage_seconds'))"

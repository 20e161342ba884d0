#!/bin/bash
# Round 6: the shader clock during the critical problem's pair loop (s_memtime / s_memrealtime).
set -o pipefail
O=gpurun_out/r6au
mkdir -p $O
for t in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_$t.json 2> $O/b_$t.err || { echo "bench failed"; tail -20 $O/b_$t.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b_$t.json').read().strip().splitlines()[-1]);print('bench $t', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['diag']['svm'].get('ws_critical'))"; done

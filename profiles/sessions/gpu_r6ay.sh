#!/bin/bash
# Round 6: the selection's phase split on the critical problem.
set -o pipefail
O=gpurun_out/r6ay
mkdir -p $O
timeout -k 10 300 python bench.py --gpus 1 --steps 10 --warmup 3 > $O/b.json 2> $O/b.err || { echo "bench failed"; tail -20 $O/b.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/b.json').read().strip().splitlines()[-1]);print('bench', d['ms_per_step'], d['diag']['svm'].get('ws_critical'))"

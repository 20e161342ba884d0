#!/bin/bash
# Round 6 (end): config 3 (1M rows, warm) on the final tree.
set -o pipefail
O=gpurun_out/r6bx
mkdir -p $O
timeout -k 10 900 python -u bench.py --rows 1000000 --steps 2 --warmup 1 > $O/cfg3.json 2> $O/cfg3.err || { echo "cfg3 failed"; tail -20 $O/cfg3.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/cfg3.json').read().strip().splitlines()[-1]);print('cfg3', d['ms_per_step'], d.get('auroc'), d.get('stage_seconds'))"

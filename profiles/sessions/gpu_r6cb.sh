#!/bin/bash
# Round 6 (end): config 4 / 5 / gbdt records on the final tree.
set -o pipefail
O=gpurun_out/r6cb
mkdir -p $O
timeout -k 10 300 python bench.py --config infer --steps 10 --warmup 3 > $O/infer.json 2> $O/infer.err || { echo "infer failed"; tail -20 $O/infer.err; exit 1; }
timeout -k 10 300 python bench.py --config gbdt --steps 10 --warmup 3 > $O/gbdt.json 2> $O/gbdt.err || { echo "gbdt failed"; tail -20 $O/gbdt.err; exit 1; }
timeout -k 10 400 python bench.py --config deep --steps 5 --warmup 2 > $O/deep.json 2> $O/deep.err || { echo "deep failed"; tail -20 $O/deep.err; exit 1; }
for c in infer gbdt deep; do python3 -c "import json;d=json.loads(open('$O/$c.json').read().strip().splitlines()[-1]);print('$c', d['ms_per_step'], d['value'], d['unit'], d.get('auroc'))"; done

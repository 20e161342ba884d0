#!/bin/bash
# Round 3 final config sweep: 5 (deep, 1000 stumps x 5 seeds), 3-GBC (gbdt), 4 (infer), headline x20.
set -o pipefail
mkdir -p gpurun_out/final
timeout -k 10 400 python3 bench.py --config deep --steps 2 --warmup 1 > gpurun_out/final/deep.json 2> gpurun_out/final/deep.err || { echo "deep failed"; tail -20 gpurun_out/final/deep.err; exit 1; }
timeout -k 10 300 python3 bench.py --config gbdt --steps 10 --warmup 3 > gpurun_out/final/gbdt.json 2> gpurun_out/final/gbdt.err || { echo "gbdt failed"; tail -20 gpurun_out/final/gbdt.err; exit 1; }
timeout -k 10 300 python3 bench.py --config infer --steps 5 --warmup 1 > gpurun_out/final/infer.json 2> gpurun_out/final/infer.err || { echo "infer failed"; tail -20 gpurun_out/final/infer.err; exit 1; }
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/head20.json 2> gpurun_out/final/head20.err || { echo "headline failed"; tail -20 gpurun_out/final/head20.err; exit 1; }
for f in deep gbdt infer head20; do python3 -c "import json; d=json.loads(open('gpurun_out/final/$f.json').read().strip().splitlines()[-1]); print('$f', d['ms_per_step'], d['value'], d['unit'], d.get('auroc'))"; done

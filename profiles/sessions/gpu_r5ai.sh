#!/bin/bash
# Round 5: headline A/B of the matrix-core KNN filter at 10k rows (forced on vs the size rule).
set -o pipefail
O=gpurun_out/r5ai
mkdir -p $O
for i in 1 2; do
  for m in auto 1; do
    HFENS_KNN_MFMA=$m timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_${m}_$i.json 2> $O/bench_${m}_$i.err || { echo "bench failed"; tail -20 $O/bench_${m}_$i.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/bench_${m}_$i.json').read().strip().splitlines()[-1]);print('$m', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"
  done
done

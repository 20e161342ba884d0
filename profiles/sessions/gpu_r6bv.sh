#!/bin/bash
# Round 6 (end): 100 timed steps of the headline on the final tree (max / median of the step times,
# VERDICT r5 #5) and the driver's 20-step command, twice.
set -o pipefail
O=gpurun_out/r6bv
mkdir -p $O
timeout -k 10 300 python bench.py --gpus 1 --steps 100 --warmup 5 > $O/b_100.json 2> $O/b_100.err || { echo "bench failed"; tail -20 $O/b_100.err; exit 1; }
python3 -c "
import json, statistics as s
d=json.loads(open('$O/b_100.json').read().strip().splitlines()[-1]); st=d['diag']['step_ms']
m=s.median(st); print('100 steps', d['ms_per_step'], 'median', m, 'max', max(st), 'max/median %.3f' % (max(st)/m), 'steps > 1.25x median:', sum(x > 1.25*m for x in st))"
for t in 1 2; do
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_$t.json 2> $O/b_$t.err || { echo "bench failed"; tail -20 $O/b_$t.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b_$t.json').read().strip().splitlines()[-1]);print('bench $t', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"; done

#!/bin/bash
# Round 6 (end): is config 3's 17.5 s (r6bx) the box or the tree?  One 1M interior-point solve timed
# (r6an measured 0.575 s on its box), then config 3 with the stacking GBC per stage (no persistent launch).
set -o pipefail
O=gpurun_out/r6by
mkdir -p $O
HFENS_IPM_CORRECTORS=2 REPS=2 timeout -k 10 300 python scripts/probes/ipm_trajectory.py 1000000 > $O/traj_c2.log 2>&1 || { echo "traj failed"; tail -20 $O/traj_c2.log; exit 1; }
tail -2 $O/traj_c2.log
HFENS_GBDT_PERSIST_STACK=0 timeout -k 10 900 python -u bench.py --rows 1000000 --steps 2 --warmup 1 > $O/cfg3_np.json 2> $O/cfg3_np.err || { echo "cfg3 failed"; tail -20 $O/cfg3_np.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/cfg3_np.json').read().strip().splitlines()[-1]);print('cfg3 persist_stack=0', d['ms_per_step'], d.get('auroc'))"

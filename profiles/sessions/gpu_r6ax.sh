#!/bin/bash
# Round 6: gradient-update workgroups of 64 rows (waves split the tiles) vs 256 rows, one box, interleaved.
set -o pipefail
O=gpurun_out/r6ax
mkdir -p $O
for R in 64 256 64b 256b; do
  export HFENS_WS_GUPDATE_RW=${R%b}
  HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 12 --warmup 3 > $O/tl_$R.json 2> $O/tl_$R.err || { echo "tl failed"; tail -20 $O/tl_$R.err; exit 1; }
  echo "rw $R: $(python3 scripts/probes/tl_summary.py $O/tl_$R.err 3 | head -1)"
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_$R.json 2> $O/b_$R.err || { echo "bench failed"; tail -20 $O/b_$R.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b_$R.json').read().strip().splitlines()[-1]);print('bench $R', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['diag']['svm']['ws_pairs_max'])"
done

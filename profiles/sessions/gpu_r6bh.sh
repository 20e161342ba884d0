#!/bin/bash
# Round 6: two working-set groups (the 10k problem | the 35 smaller ones), the second on the normal-priority
# svc_ws_1 stream (HFENS_SVM_WS_GROUPS=2 HFENS_SVM_WS_LAST_SIDE=1) vs three groups (default).
set -o pipefail
O=gpurun_out/r6bh
mkdir -p $O
for P in g3 g2 g3b g2b; do
  case $P in g3*) export HFENS_SVM_WS_GROUPS=3 HFENS_SVM_WS_LAST_SIDE=0;; *) export HFENS_SVM_WS_GROUPS=2 HFENS_SVM_WS_LAST_SIDE=1;; esac
  HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 12 --warmup 3 > $O/tl_$P.json 2> $O/tl_$P.err || { echo "tl failed"; tail -20 $O/tl_$P.err; exit 1; }
  echo "prio $P: $(python3 scripts/probes/tl_summary.py $O/tl_$P.err 3 | head -1)"
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_$P.json 2> $O/b_$P.err || { echo "bench failed"; tail -20 $O/b_$P.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b_$P.json').read().strip().splitlines()[-1]);print('bench $P', d['ms_per_step'], d['diag']['step_ms_min_med_max'])"
done

#!/bin/bash
# Round 6: the stacking GBC as per-stage launches (HFENS_GBDT_PERSIST_STACK=0) vs one persistent launch:
# does the persistent kernel hold the CUs the SMO's solve workgroups need?
set -o pipefail
O=gpurun_out/r6bi
mkdir -p $O
for P in p1 p0 p1b p0b; do
  case $P in p1*) export HFENS_GBDT_PERSIST_STACK=1;; *) export HFENS_GBDT_PERSIST_STACK=0;; esac
  HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 12 --warmup 3 > $O/tl_$P.json 2> $O/tl_$P.err || { echo "tl failed"; tail -20 $O/tl_$P.err; exit 1; }
  echo "prio $P: $(python3 scripts/probes/tl_summary.py $O/tl_$P.err 3 | head -1)"
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_$P.json 2> $O/b_$P.err || { echo "bench failed"; tail -20 $O/b_$P.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b_$P.json').read().strip().splitlines()[-1]);print('bench $P', d['ms_per_step'], d['diag']['step_ms_min_med_max'])"
done

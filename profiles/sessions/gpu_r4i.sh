#!/bin/bash
# round 4: lean inner solver vs classic: per-pair cost (ws_stats, sequential bases) and the headline
set -o pipefail
D=gpurun_out/r4i
mkdir -p $D
for k in lean classic; do
  HFENS_SVM_WS_PAIRS=$k HFENS_CONCURRENT_BASES=0 timeout -k 10 300 python scripts/ws_stats.py > $D/ws_stats_$k.log 2>&1 || { echo "ws_stats failed"; tail -30 $D/ws_stats_$k.log; exit 1; }
  echo $k; grep -v amdgpu.ids $D/ws_stats_$k.log | tail -6
done
run() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $D/$name.json 2> $D/$name.err || { echo "$name failed"; tail -30 $D/$name.err; return 1; }
  python -c "import json; d=json.loads(open('$D/$name.json').read().strip().split('\n')[-1]); print('$name', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'], d['diag']['svm'])"
}
run classic HFENS_SVM_WS_PAIRS=classic

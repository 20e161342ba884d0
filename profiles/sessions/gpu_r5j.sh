#!/bin/bash
# Round 5: cascade part budget sweep (rounds × part eps) — timelines, per-problem stats, bench.
set -o pipefail
O=gpurun_out/r5j
mkdir -p $O
run() {  # run TAG ENV...
  local tag=$1; shift
  env "$@" HFENS_TRACE_DEV=1 timeout -k 10 200 python bench.py --steps 8 --warmup 3 > $O/tl_$tag.json 2> $O/tl_$tag.err || { echo "$tag failed"; tail -20 $O/tl_$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.loads(open('$O/tl_$tag.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['auroc'], d['diag']['step_ms_min_med_max'])")"
  grep "^\[dev\]" $O/tl_$tag.err | tail -2 | head -1 | cut -c1-200
}
run r12 HFENS_SVM_CASCADE_ROUNDS=12
run r8 HFENS_SVM_CASCADE_ROUNDS=8
run r20 HFENS_SVM_CASCADE_ROUNDS=20
run r12e03 HFENS_SVM_CASCADE_ROUNDS=12 HFENS_SVM_CASCADE_EPS=0.03
run r8p1600 HFENS_SVM_CASCADE_ROUNDS=8 HFENS_SVM_CASCADE_PART=1600
run r12p800 HFENS_SVM_CASCADE_ROUNDS=12 HFENS_SVM_CASCADE_PART=800
run cold HFENS_SVM_CASCADE=0
timeout -k 10 200 python scripts/ws_stats.py > $O/ws_stats.log 2>&1 && grep -E "^cascade|^q |^inner|problem" $O/ws_stats.log | head -8
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print('bench', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"

#!/bin/bash
# Round 6: cascade-seed parameters for the headline's critical problem, same box.
set -o pipefail
O=gpurun_out/r6v
mkdir -p $O
run() {  # run TAG ENV...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_$tag.json 2> $O/b_$tag.err || { echo "$tag failed"; tail -20 $O/b_$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'], d['diag']['svm'].get('ws_rounds_max'), d['diag']['svm'].get('ws_pairs_max'))")"
}
run base && run r6 HFENS_SVM_CASCADE_ROUNDS=6 && run r4 HFENS_SVM_CASCADE_ROUNDS=4 && run r6e03 HFENS_SVM_CASCADE_ROUNDS=6 HFENS_SVM_CASCADE_EPS=0.3 && run e03 HFENS_SVM_CASCADE_EPS=0.3 && run r5 HFENS_SVM_CASCADE_ROUNDS=5 && run base2 && run r6b HFENS_SVM_CASCADE_ROUNDS=6 && run r6e03b HFENS_SVM_CASCADE_ROUNDS=6 HFENS_SVM_CASCADE_EPS=0.3 && run r4b HFENS_SVM_CASCADE_ROUNDS=4

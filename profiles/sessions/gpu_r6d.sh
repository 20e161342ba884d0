#!/bin/bash
# Round 6: hardware-queue sharing matrix of the fit's streams; ordering A/B on one box.
set -o pipefail
O=gpurun_out/r6d
mkdir -p $O
timeout -k 10 120 python scripts/probes/hwq_probe.py > $O/hwq.log 2>&1 || { echo "probe failed"; tail -20 $O/hwq.log; exit 1; }
cat $O/hwq.log
run() {  # run TAG ENV...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_$tag.json 2> $O/b_$tag.err || { echo "$tag failed"; tail -20 $O/b_$tag.err; exit 1; }
  echo "$tag $(python3 -c "import json;d=json.loads(open('$O/b_$tag.json').read().strip().splitlines()[-1]);print(d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])")"
}
run after && run before HFENS_BASES_AFTER_CV=0 && run r5flow HFENS_LASSO_EARLY_SPEC=0 HFENS_PRELAUNCH_BASES=0 && run after2 && run before2 HFENS_BASES_AFTER_CV=0

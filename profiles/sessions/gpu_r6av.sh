#!/bin/bash
# Round 6: the no-op rounds after convergence — seeded rounds enqueued ahead 48 (default) vs 32 vs 28:
# traced medians (SMO done, stack_fit) and bench.
set -o pipefail
O=gpurun_out/r6av
mkdir -p $O
for A in 48 32 28 48b; do
  export HFENS_SVM_WS_SEEDED_AHEAD=${A%b}
  HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 12 --warmup 3 > $O/tl_$A.json 2> $O/tl_$A.err || { echo "tl failed"; tail -20 $O/tl_$A.err; exit 1; }
  echo "ahead $A: $(python3 scripts/probes/tl_summary.py $O/tl_$A.err 3 | head -2 | tr '\n' ' ')"
  timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_$A.json 2> $O/b_$A.err || { echo "bench failed"; tail -20 $O/b_$A.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b_$A.json').read().strip().splitlines()[-1]);print('bench $A', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['diag']['svm']['ws_rounds_max'])"
done

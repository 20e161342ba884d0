#!/bin/bash
# Round 6: cost of the timed steps' stage-timing events (bench.py HFENS_BENCH_STAGE_EVENTS), A/B
# interleaved on one box, 3 runs each.
set -o pipefail
O=gpurun_out/r6bt
mkdir -p $O
for r in a b c; do for v in 1 0; do
  HFENS_BENCH_STAGE_EVENTS=$v timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_${v}$r.json 2> $O/b_${v}$r.err || { echo "bench failed"; tail -20 $O/b_${v}$r.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/b_${v}$r.json').read().strip().splitlines()[-1]);print('events=$v ($r)', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['diag']['host_cpu_fraction'], d['diag']['busiest_threads_cpu_s'])"
done; done

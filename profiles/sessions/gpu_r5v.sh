#!/bin/bash
# Round 5: bimodal step times after the plan thread / event reads — A/B with timelines.
set -o pipefail
O=gpurun_out/r5v
mkdir -p $O
b() {  # b TAG ENV...
  local tag=$1; shift
  env "$@" timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_$tag.json 2> $O/bench_$tag.err || { echo "bench $tag failed"; tail -5 $O/bench_$tag.err; exit 1; }
  python3 -c "import json;d=json.loads(open('$O/bench_$tag.json').read().strip().splitlines()[-1]);print('bench $tag', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"
}
b thread
b nothread HFENS_PLAN_THREAD=0
b thread2
b nothread2 HFENS_PLAN_THREAD=0
HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 8 --warmup 3 > $O/tl.json 2> $O/tl.err || { echo "tl failed"; tail -20 $O/tl.err; exit 1; }
grep -E "^\[dev\]" $O/tl.err | tail -8 | cut -c1-330

#!/bin/bash
# Quick headline check: the driver's bench command twice, then a host-timeline trace run.
set -o pipefail
D=gpurun_out/quick
mkdir -p $D
for k in 1 2; do
  timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench$k.json 2> $D/bench$k.err \
    || { echo "bench failed"; tail -30 $D/bench$k.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench$k.json')); print('bench$k', d['ms_per_step'], d['config']['stage_seconds'], d['diag']['step_ms_min_med_max'], d['diag']['svm'])"
done
HFENS_TRACE_HOST=1 timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 4 --warmup 2 > $D/trace.json 2> $D/trace.err \
  || { echo "trace failed"; tail -30 $D/trace.err; exit 1; }
grep "\[host\]" $D/trace.err | tail -3

#!/bin/bash
# round 4: device timeline of the headline fit (HFENS_TRACE_DEV device events + host marks, no
# profiler attached) — where the SVC's post-SMO tail goes
set -o pipefail
D=gpurun_out/r4s
mkdir -p $D
HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 6 --warmup 2 > $D/trace.json 2> $D/trace.err || { echo "trace failed"; tail -30 $D/trace.err; exit 1; }
grep -E "^\[(dev|host)\]" $D/trace.err | tail -6

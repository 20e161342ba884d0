#!/bin/bash
# round 4: host marks between the LassoCV result and the SMO launch
set -o pipefail
D=gpurun_out/r4ac
mkdir -p $D
HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 4 --warmup 2 > $D/trace.json 2> $D/trace.err || { echo "trace failed"; tail -30 $D/trace.err; exit 1; }
grep -E "^\[(dev|host)\]" $D/trace.err | tail -2

#!/bin/bash
# round 4: LassoCV path alone vs inside the fit (device marks)
set -o pipefail
D=gpurun_out/r4z
mkdir -p $D
timeout -k 10 200 python -u scripts/probes/lasso_probe.py > $D/lasso_probe.log 2>&1 || { echo "probe failed"; tail -30 $D/lasso_probe.log; exit 1; }
grep spec $D/lasso_probe.log
HFENS_TRACE_DEV=1 timeout -k 10 200 python bench.py --steps 4 --warmup 2 > $D/trace.json 2> $D/trace.err || { echo "trace failed"; tail -30 $D/trace.err; exit 1; }
grep -E "^\[dev\]" $D/trace.err | tail -3

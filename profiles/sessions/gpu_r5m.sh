#!/bin/bash
set -o pipefail
O=gpurun_out/r5m
mkdir -p $O
export HFENS_SVM_CASCADE_ROUNDS=8 HFENS_SVM_CASCADE_PART=1600
timeout -k 10 300 python scripts/probes/sync_debug.py > $O/sync.log 2>&1 || { echo "sync probe failed"; tail -20 $O/sync.log; exit 1; }
grep -v amdgpu.ids $O/sync.log | cut -c1-330 | tail -60
HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 8 --warmup 3 > $O/tl.json 2> $O/tl.err || { echo "tl failed"; tail -20 $O/tl.err; exit 1; }
grep "^\[host\]" $O/tl.err | tail -2 | head -1 | tr ' ' '\n' | grep -v ws_chunk | tr '\n' ' ' | cut -c1-1400; echo

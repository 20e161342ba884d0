#!/bin/bash
# Round 5: where the host blocks (cProfile of 3 steps) + host/device timeline with the new marks.
set -o pipefail
O=gpurun_out/r5l
mkdir -p $O
export HFENS_SVM_CASCADE_ROUNDS=8 HFENS_SVM_CASCADE_PART=1600
timeout -k 10 300 python scripts/probes/host_profile.py > $O/host_profile.log 2>&1 || { echo "profile failed"; tail -20 $O/host_profile.log; exit 1; }
head -60 $O/host_profile.log | cut -c1-200
HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 8 --warmup 3 > $O/tl.json 2> $O/tl.err || { echo "tl failed"; tail -20 $O/tl.err; exit 1; }
grep "^\[dev\]" $O/tl.err | tail -2 | head -1 | cut -c1-400
grep "^\[host\]" $O/tl.err | tail -2 | head -1 | tr ' ' '\n' | grep -v ws_chunk | tr '\n' ' ' | cut -c1-1200; echo

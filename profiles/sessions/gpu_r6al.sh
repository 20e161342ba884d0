#!/bin/bash
# Round 6: the fit's tail after the SMO — host marks between the LassoCV's read and the stack's reads.
set -o pipefail
O=gpurun_out/r6al
mkdir -p $O
HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 8 --warmup 3 > $O/tl.json 2> $O/tl.err || { echo "tl failed"; tail -20 $O/tl.err; exit 1; }
for i in 4 3 2; do grep "^\[dev\]" $O/tl.err | tail -$i | head -1 | cut -c1-900; grep "^\[host\]" $O/tl.err | tail -$i | head -1 | tr " " "\n" | grep -v ws_chunk | tr "\n" " " | cut -c1-1500; echo; done

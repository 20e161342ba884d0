#!/bin/bash
set -o pipefail
O=gpurun_out/r6aa
mkdir -p $O
HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 8 --warmup 3 > $O/tl.json 2> $O/tl.err || { echo "tl failed"; tail -20 $O/tl.err; exit 1; }
grep "^\[dev\]" $O/tl.err | tail -3 | head -2 | cut -c1-900
grep "^\[host\]" $O/tl.err | tail -3 | head -2 | tr ' ' '\n' | grep -v ws_chunk | tr '\n' ' ' | cut -c1-2000; echo

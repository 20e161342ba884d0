#!/bin/bash
set -o pipefail
D=gpurun_out/hmarks
mkdir -p $D
HFENS_TRACE_HOST=1 timeout -k 10 300 python bench.py --steps 3 --warmup 2 > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -30 $D/bench.err; exit 1; }
grep "^\[host\]" $D/bench.err | tail -3

#!/bin/bash
# Round 6 (end): kernel stats of the headline on the final tree (rocprofv3 --kernel-trace --stats), 5 timed steps.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
O=gpurun_out/r6bj
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof -o run -- python3 bench.py --steps 5 --warmup 3 > $O/bench.json 2> $O/prof.err || { echo "prof failed"; tail -20 $O/prof.err; exit 1; }
ls $O/prof

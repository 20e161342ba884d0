#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/prof_ws
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ws -o ws --output-format csv -- python scripts/ws_diag.py ws:0.1 > gpurun_out/prof_ws.log 2>&1 || { echo "rocprof failed"; tail -20 gpurun_out/prof_ws.log; exit 1; }
tail -5 gpurun_out/prof_ws.log

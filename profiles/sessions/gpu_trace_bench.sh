#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
rm -rf gpurun_out/trace_bench
timeout -k 10 400 rocprofv3 --kernel-trace -d gpurun_out/trace_bench -o tb --output-format csv -- python bench.py --steps 3 --warmup 2 > gpurun_out/trace_bench.log 2>&1 || { tail -20 gpurun_out/trace_bench.log; exit 1; }

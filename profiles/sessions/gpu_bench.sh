#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --steps 5 --warmup 2 --timings > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
grep -v amdgpu.ids gpurun_out/bench.err; cat gpurun_out/bench.json
HFENS_CONCURRENT_BASES=0 timeout -k 10 300 python bench.py --steps 5 --warmup 2 > gpurun_out/bench_seq.json 2> gpurun_out/bench_seq.err || { tail -20 gpurun_out/bench_seq.err; exit 1; }
cat gpurun_out/bench_seq.json

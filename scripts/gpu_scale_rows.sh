#!/bin/bash
# Full-ensemble development fit at growing row counts (cfg 3 path): per-stage timings.
set -o pipefail
mkdir -p gpurun_out/rows
timeout -k 10 300 python bench.py --rows 30000 --steps 1 --warmup 1 --timings > gpurun_out/rows/r30k.json 2> gpurun_out/rows/r30k.err || { echo "30k failed"; tail -20 gpurun_out/rows/r30k.err; exit 1; }
grep -v amdgpu.ids gpurun_out/rows/r30k.err; cat gpurun_out/rows/r30k.json
HFENS_SVM_SOLVER=ws timeout -k 10 300 python bench.py --rows 30000 --steps 1 --warmup 0 --timings > gpurun_out/rows/r30k_ws.json 2> gpurun_out/rows/r30k_ws.err || { echo "30k ws failed"; tail -20 gpurun_out/rows/r30k_ws.err; exit 1; }
grep -v amdgpu.ids gpurun_out/rows/r30k_ws.err; cat gpurun_out/rows/r30k_ws.json
HFENS_SVM_SOLVER=ws timeout -k 10 500 python bench.py --rows 100000 --steps 1 --warmup 0 --timings > gpurun_out/rows/r100k_ws.json 2> gpurun_out/rows/r100k_ws.err || { echo "100k ws failed"; tail -20 gpurun_out/rows/r100k_ws.err; exit 1; }
grep -v amdgpu.ids gpurun_out/rows/r100k_ws.err; cat gpurun_out/rows/r100k_ws.json

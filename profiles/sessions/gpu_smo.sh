#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_train_gpu.py tests/test_checkpoint.py -x -q -k "svc or libsvm" > gpurun_out/pytest_smo.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_smo.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_smo.log; exit 1; }
timeout -k 10 300 python scripts/ws_diag.py exact > gpurun_out/ws_diag.log 2>&1 || { tail -20 gpurun_out/ws_diag.log; exit 1; }
grep -v amdgpu.ids gpurun_out/ws_diag.log
timeout -k 10 300 python bench.py --steps 3 --warmup 1 --timings > gpurun_out/bench.json 2> gpurun_out/bench.err || { tail -20 gpurun_out/bench.err; exit 1; }
grep -v amdgpu.ids gpurun_out/bench.err; cat gpurun_out/bench.json

#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_train_gpu.py -x -q > gpurun_out/pytest_train.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_train.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_train.log; exit 1; }
timeout -k 10 300 python bench.py --config gbdt --steps 3 --warmup 1 > gpurun_out/bench_gbdt.json 2> gpurun_out/bench_gbdt.err || { tail -20 gpurun_out/bench_gbdt.err; exit 1; }
cat gpurun_out/bench_gbdt.json
timeout -k 10 600 python bench.py --config deep --steps 1 --warmup 1 > gpurun_out/bench_deep.json 2> gpurun_out/bench_deep.err || { tail -20 gpurun_out/bench_deep.err; exit 1; }
cat gpurun_out/bench_deep.json

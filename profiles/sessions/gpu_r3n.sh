#!/bin/bash
# Round 3: the GBDT stage counter advanced inside the partial-reduce launch: GBDT GPU tests, the
# shard-size stage-cost probe, the 3-GBC bench.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py -x -q -k "gbdt or gbc or stage" --timeout 200 --timeout-method thread -p no:cacheprovider > gpurun_out/r3n_pytest.log 2>&1 || { echo "pytest failed"; tail -40 gpurun_out/r3n_pytest.log; exit 1; }
tail -2 gpurun_out/r3n_pytest.log
timeout -k 10 300 python3 -u scripts/probes/gbdt_shard_probe.py > gpurun_out/r3n_shard.log 2>&1 || { echo "probe failed"; tail -20 gpurun_out/r3n_shard.log; exit 1; }
grep -v amdgpu.ids gpurun_out/r3n_shard.log | grep -v "^{"
timeout -k 10 300 python3 -u bench.py --config gbdt --steps 10 --warmup 3 > gpurun_out/r3n_gbdt.json 2> gpurun_out/r3n_gbdt.err || { echo "gbdt bench failed"; tail -20 gpurun_out/r3n_gbdt.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r3n_gbdt.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d.get('auroc'))"

#!/bin/bash
# Round 5: GBDT stage — parallel prologue, MFMA sums folded once, wide features over all waves.
set -o pipefail
O=gpurun_out/r5x
mkdir -p $O
#timeout -k 10 600 python -u -m pytest tests/test_train_gpu.py tests/test_bench_parity_gpu.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider -k "gbdt or gbc or stump or bench_parity" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
#tail -2
timeout -k 10 300 python scripts/probes/gbdt_stage_phases.py > $O/phases.log 2>&1 || { echo "phases failed"; tail -20 $O/phases.log; exit 1; }
grep -v amdgpu.ids $O/phases.log
PROBE_ROWS=125000 timeout -k 10 300 python scripts/probes/gbdt_stage_phases.py > $O/phases_125k.log 2>&1 || { echo "phases failed"; tail -20 $O/phases_125k.log; exit 1; }
grep -v amdgpu.ids $O/phases_125k.log
timeout -k 10 300 python bench.py --config gbdt > $O/bench_gbdt.json 2> $O/bench_gbdt.err || { echo "bench gbdt failed"; tail -5 $O/bench_gbdt.err; exit 1; }
cut -c1-200 $O/bench_gbdt.json

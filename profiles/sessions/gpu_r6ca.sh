#!/bin/bash
# Round 6: the whole GPU suite + smoke + headline bench on the current tree (late round).
set -o pipefail
O=gpurun_out/r6ca
mkdir -p $O
timeout -k 10 500 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "xgmi or probe or dp_stage or data_parallel or task_policy" > $O/pytest_mp.log 2>&1 || { echo "pytest mp failed"; tail -60 $O/pytest_mp.log; exit 1; }
tail -2 $O/pytest_mp.log
timeout -k 10 1000 python -u -m pytest tests -m gpu -q --timeout 200 --timeout-method thread -p no:cacheprovider --deselect tests/test_train_gpu.py::test_gbdt_stage_data_parallel_bit_identical > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest_gpu.log; exit 1; }
tail -2 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print('bench', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"

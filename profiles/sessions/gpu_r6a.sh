#!/bin/bash
# Round 6 first call: ADVICE-r5 fixes (probe lock-step tests, early-read-off test), the GPU suite,
# smoke, the headline bench and a device/host timeline of the headline.
set -o pipefail
O=gpurun_out/r6a
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_train_gpu.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider -k "xgmi or probe or dp_stage or data_parallel or early_read" > $O/pytest_mp.log 2>&1 || { echo "pytest mp failed"; tail -60 $O/pytest_mp.log; exit 1; }
tail -3 $O/pytest_mp.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 180 --timeout-method thread -p no:cacheprovider --deselect tests/test_train_gpu.py::test_gbdt_stage_data_parallel_bit_identical > $O/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest_gpu.log; exit 1; }
tail -3 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $O/smoke.log; exit 1; }
tail -2 $O/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo "bench failed"; tail -5 $O/bench.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/bench.json').read().strip().splitlines()[-1]);print('bench', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"
HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 8 --warmup 3 > $O/tl.json 2> $O/tl.err || { echo "tl failed"; tail -20 $O/tl.err; exit 1; }
grep "^\[dev\]" $O/tl.err | tail -2 | head -1 | cut -c1-900
grep "^\[host\]" $O/tl.err | tail -2 | head -1 | tr ' ' '\n' | grep -v ws_chunk | tr '\n' ' ' | cut -c1-1500; echo

#!/bin/bash
# Round 6: after breaking the SMO state's reference cycles — cycle probe, outliers (GC on / off), bench.
set -o pipefail
O=gpurun_out/r6q
mkdir -p $O
timeout -k 10 200 python scripts/probes/cycle_probe.py > $O/cycles.log 2>&1 && grep -v amdgpu.ids $O/cycles.log | head -8
SYNC=0 timeout -k 10 300 python scripts/probes/step_outliers.py 150 > $O/out_gc_on.log 2>&1 && tail -1 $O/out_gc_on.log | cut -c1-1500
SYNC=0 GC_OFF=1 timeout -k 10 300 python scripts/probes/step_outliers.py 150 > $O/out_gc_off.log 2>&1 && tail -1 $O/out_gc_off.log | cut -c1-1500
timeout -k 10 300 python -u -m pytest tests/test_svm_ws_gpu.py tests/test_train_gpu.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider -k "ws or prelaunch or svc" > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -60 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
for t in a b; do timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/b_$t.json 2> $O/b_$t.err || { echo "bench failed"; tail -20 $O/b_$t.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/b_$t.json').read().strip().splitlines()[-1]);print('bench', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"; done

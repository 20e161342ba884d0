#!/bin/bash
# Round 5: native f64 Gram from the f32 copy of Φ as the interior point's default — tests, config 3.
set -o pipefail
O=gpurun_out/r5ao
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_linalg_gpu.py tests/test_svc_scale_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
tail -2 $O/pytest.log
timeout -k 10 900 python -u bench.py --rows 1000000 --steps 2 --warmup 1 > $O/fullstack_1m.json 2> $O/fullstack_1m.err || { echo "1m failed"; tail -20 $O/fullstack_1m.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/fullstack_1m.json').read().strip().splitlines()[-1]);print('1M', d['ms_per_step'], d['auroc'], d['diag'].get('step_ms_min_med_max'), d['config'].get('stage_seconds'), d['diag']['svm'].get('lowrank',{}).get('ipm_iters'))"

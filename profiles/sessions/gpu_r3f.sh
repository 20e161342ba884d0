#!/bin/bash
# Round 3: fp8 forest (depth-templated walks) tests + config 5 rates; headline host marks.
set -o pipefail
D=gpurun_out/r3f
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_forest_fp8_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 300 python3 -u bench.py --config deep --steps 3 --warmup 1 > $D/deep.json 2> $D/deep.err || { echo "deep failed"; tail -30 $D/deep.err; exit 1; }
python3 -c "import json; d=json.loads(open('$D/deep.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['infer_rows_x_models_per_sec'], d['fp8_leaf_inference'])"
timeout -k 10 300 python3 -u bench.py --config deep --depth 3 --trees 300 --steps 2 --warmup 1 > $D/deep3.json 2> $D/deep3.err || { echo "deep3 failed"; tail -30 $D/deep3.err; exit 1; }
python3 -c "import json; d=json.loads(open('$D/deep3.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['auroc'], d['fp8_leaf_inference'])"
HFENS_TRACE_HOST=1 timeout -k 10 300 python bench.py --steps 5 --warmup 2 > $D/hmarks.json 2> $D/hmarks.err || { echo "marks failed"; tail -30 $D/hmarks.err; exit 1; }
grep "^\[host\]" $D/hmarks.err | tail -1

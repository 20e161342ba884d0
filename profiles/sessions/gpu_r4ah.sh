#!/bin/bash
# round 4: decision-kernel K-step count matched to F = 17 (KS = 9) — SVC tests, kernel stats
set -o pipefail
D=gpurun_out/r4ah
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_svm_ws_gpu.py tests/test_train_gpu.py tests/test_infer_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "svc or svm or platt or oof or rbf or ws" > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
R=$PWD
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o hb --output-format csv -- python bench.py --steps 5 --warmup 2 > $D/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $D/prof.log; exit 1; }
f=$(find $D/prof -name "*kernel_stats.csv" | head -1)
cp $f $D/kernel_stats.csv
python - <<'PY'
import csv
r = list(csv.reader(open("gpurun_out/r4ah/kernel_stats.csv")))
for x in r[1:]:
    if any(k in x[0] for k in ("svm_dec_batch", "platt", "svc_oof")):
        print(x[0][:50], x[1], round(float(x[3]) / 1e3, 1), "us avg", round(float(x[5]) / 1e3, 1), round(float(x[6]) / 1e3, 1))
PY

#!/bin/bash
# Lock-step decoupling of the working-set SMO: largest problems on their own stream.
set -o pipefail
D=gpurun_out/wssplit
rm -rf $D; mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_svm_ws_gpu.py tests/test_train_gpu.py -x -q -k "ws or svc or stack" --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for sp in 1 2 3; do
  HFENS_SVM_WS_GROUPS=$sp timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $D/bench_$sp.json 2>$D/bench_$sp.err || { echo "bench failed"; tail $D/bench_$sp.err; exit 1; }
  python -c "import json;d=json.load(open('$D/bench_$sp.json'));print('split $sp', d['ms_per_step'], d['auroc'], d['config']['stage_seconds'], d['diag']['svm'])"
done
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/raw -o tl -- python bench.py --steps 2 --warmup 2 > $D/trace.log 2>&1 || { echo "trace failed"; tail -20 $D/trace.log; exit 1; }
f=$(find $D/raw -name "*kernel_trace.csv" | head -1)
python scripts/fit_timeline.py "$f" > $D/timeline.txt && head -30 $D/timeline.txt
rm -rf $D/raw

#!/bin/bash
set -o pipefail
D=gpurun_out/fittl
rm -rf $D; mkdir -p $D
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $D/raw -o tl -- python bench.py --steps 2 --warmup 2 > $D/bench.log 2>&1 || { echo "trace failed"; tail -20 $D/bench.log; exit 1; }
f=$(find $D/raw -name "*kernel_trace.csv" | head -1)
python scripts/fit_timeline.py "$f" > $D/timeline.txt && cat $D/timeline.txt
rm -rf $D/raw
for fr in 0.2 0.3; do
  HFENS_SVM_WS_FRAC=$fr timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $D/bench_frac$fr.json 2>/dev/null || { echo "bench failed"; exit 1; }
  python -c "import json;d=json.load(open('$D/bench_frac$fr.json'));print('frac $fr', d['ms_per_step'], d['auroc'], d['diag']['svm'])"
done

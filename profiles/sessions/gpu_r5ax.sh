#!/bin/bash
# Round 5: matrix-core KNN filter as the default from 4k x 4k pairs: tests, probe, headline A/B.
set -o pipefail
O=gpurun_out/r5ax
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_prep_gpu.py tests/test_bench_parity_gpu.py -x -q --timeout 180 --timeout-method thread -p no:cacheprovider > $O/pytest_prep.log 2>&1 || { echo "pytest prep failed"; tail -40 $O/pytest_prep.log; exit 1; }
tail -2 $O/pytest_prep.log
timeout -k 10 300 python scripts/probes/knn_mfma_probe.py 10000 50000 100000 300000 > $O/probe.log 2>&1 || { echo "probe failed"; tail -20 $O/probe.log; exit 1; }
grep -v amdgpu.ids $O/probe.log | grep mfma
for i in 1 2; do
  for m in auto 0; do
    HFENS_KNN_MFMA=$m timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $O/bench_${m}_$i.json 2> $O/bench_${m}_$i.err || { echo "bench failed"; tail -20 $O/bench_${m}_$i.err; exit 1; }
    python3 -c "import json;d=json.loads(open('$O/bench_${m}_$i.json').read().strip().splitlines()[-1]);print('$m', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"
  done
done

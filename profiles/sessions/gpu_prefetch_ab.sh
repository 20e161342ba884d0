#!/bin/bash
# A/B of the cooperative SMO's L2 row prefetch: equivalence tests, phase counters, driver bench.
set -o pipefail
D=gpurun_out/pf
mkdir -p $D
timeout -k 10 300 python3 -u -m pytest tests/test_train_gpu.py -k "coop" -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1 \
  || { echo "pytest failed"; tail -30 $D/pytest.log; exit 1; }
tail -1 $D/pytest.log
for pf in 0 1; do
  HFENS_SMO_PREFETCH=$pf timeout -k 10 200 python3 -u scripts/coop_phases.py > $D/phases$pf.log 2>&1 || { echo "phases failed"; tail -20 $D/phases$pf.log; exit 1; }
  echo "prefetch=$pf"; cat $D/phases$pf.log
done
for pf in 1 0 1; do
  HFENS_SMO_PREFETCH=$pf timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench$pf.json 2> $D/bench$pf.err \
    || { echo "bench failed"; tail -30 $D/bench$pf.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/bench$pf.json')); print('prefetch=$pf', d['ms_per_step'], d['config']['stage_seconds'], d['diag']['step_ms_min_med_max'])"
done

#!/bin/bash
# round 4: KNN refine spread over ≥ 2048 workgroups — KNN tests, headline bench (+ big-group inner
# stop 0.3), host/device timeline, kernel stats
set -o pipefail
D=gpurun_out/r4n
mkdir -p $D
timeout -k 10 300 python -u -m pytest tests/test_prep_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k knn > $D/pytest_knn.log 2>&1 || { echo "pytest knn failed"; tail -40 $D/pytest_knn.log; exit 1; }
tail -2 $D/pytest_knn.log
run() {
  local name=$1; shift
  env "$@" timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $D/$name.json 2> $D/$name.err || { echo "$name failed"; tail -30 $D/$name.err; return 1; }
  python -c "import json; d=json.loads(open('$D/$name.json').read().strip().split('\n')[-1]); print('$name', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'], d['diag']['svm'].get('ws_rounds_max'), d['diag']['svm'].get('ws_pairs_max'))"
}
run base HFENS_X=0 &&

run knn_f32 HFENS_KNN_EXACT=0 &&
HFENS_TRACE_HOST=1 timeout -k 10 200 python -u scripts/probes/ws_events.py > $D/ev_host.log 2>&1 || { echo "events failed"; tail -30 $D/ev_host.log; exit 1; }
tail -5 $D/ev_host.log
R=$PWD
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o hb --output-format csv -- python bench.py --steps 5 --warmup 2 > $D/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $D/prof.log; exit 1; }
f=$(find $D/prof -name "*kernel_stats.csv" | head -1)
cut -c1-120 $f > $D/kstats_short.txt; tail -n +1 $D/kstats_short.txt | sed -n 1,16p

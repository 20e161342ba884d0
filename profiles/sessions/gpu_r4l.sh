#!/bin/bash
# round 4: f64-exact KNN donors; device-side SVC OOF column — GPU tests, headline bench, aligned host/device timeline
set -o pipefail
D=gpurun_out/r4l
mkdir -p $D
echo skip-prep

echo skip-chol

timeout -k 10 560 python -u -m pytest tests/test_train_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider -k "device_svc_oof" > $D/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $D/pytest.log; exit 1; }
tail -3 $D/pytest.log
for k in 1 0; do
  HFENS_DEVICE_SVC_OOF=$k timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $D/bench_oof$k.json 2> $D/bench_oof$k.err || { echo "bench failed"; tail -30 $D/bench_oof$k.err; exit 1; }
  python -c "import json; d=json.loads(open('$D/bench_oof$k.json').read().strip().split('\n')[-1]); print('oof$k', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'])"
done
HFENS_SVM_WS_FRAC_BIG=0.3 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $D/bench_fracbig.json 2> $D/bench_fracbig.err || { echo "bench fracbig failed"; tail -30 $D/bench_fracbig.err; exit 1; }
python -c "import json; d=json.loads(open('$D/bench_fracbig.json').read().strip().split('\n')[-1]); print('fracbig0.3', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'], d['diag']['svm'])"
HFENS_SVM_WS_Q=512 timeout -k 10 200 python bench.py --steps 20 --warmup 5 > $D/bench_q512.json 2> $D/bench_q512.err || { echo "bench q512 failed"; tail -30 $D/bench_q512.err; exit 1; }
python -c "import json; d=json.loads(open('$D/bench_q512.json').read().strip().split('\n')[-1]); print('q512', d['ms_per_step'], d['diag']['step_ms_min_med_max'], d['auroc'], d['diag']['svm'])"
HFENS_TRACE_HOST=1 timeout -k 10 200 python -u scripts/probes/ws_events.py > $D/ev_host.log 2>&1 || { echo "events failed"; tail -30 $D/ev_host.log; exit 1; }
tail -6 $D/ev_host.log
timeout -k 10 200 python -u scripts/probes/ipm_probe.py 1000000 512 ipm-only f32-only > $D/ipm_mw.log 2>&1 || { echo "ipm mw failed"; tail -20 $D/ipm_mw.log; exit 1; }
cat $D/ipm_mw.log
HFENS_CHOL_MW=0 timeout -k 10 200 python -u scripts/probes/ipm_probe.py 1000000 512 ipm-only f32-only > $D/ipm_1wg.log 2>&1 || { echo "ipm 1wg failed"; tail -20 $D/ipm_1wg.log; exit 1; }
cat $D/ipm_1wg.log
R=$PWD
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $D/prof -o hb --output-format csv -- python bench.py --steps 5 --warmup 2 > $D/prof.log 2>&1 || { echo "rocprof failed"; tail -20 $D/prof.log; exit 1; }
f=$(find $D/prof -name "*kernel_stats.csv" | head -1)
head -25 $f

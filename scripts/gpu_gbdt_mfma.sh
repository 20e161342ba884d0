#!/bin/bash
# GBDT stage kernel: i8-MFMA histogram vs int64 VALU sums (HFENS_GBDT_MFMA), tests first.
set -o pipefail
D=gpurun_out/gbmf
mkdir -p $D
timeout -k 10 300 python3 -u -m pytest tests/test_train_gpu.py -x -q -k "gbdt or gbc or stump or binned" --timeout 120 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1 \
  || { echo "pytest failed"; tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
for mf in ${MFS:-1 0}; do
  export HFENS_SG_THREADS=${NT:-512}
  HFENS_GBDT_MFMA=$mf timeout -k 10 200 python3 -u bench.py --config gbdt --steps 10 --warmup 2 > $D/gbdt_$mf.json 2> $D/gbdt_$mf.err || { echo "gbdt $mf failed"; tail -20 $D/gbdt_$mf.err; exit 1; }
  HFENS_GBDT_MFMA=$mf timeout -k 10 300 python3 -u bench.py --config deep --steps 2 --warmup 1 --subsample 0.8 > $D/deep_$mf.json 2> $D/deep_$mf.err || { echo "deep $mf failed"; tail -20 $D/deep_$mf.err; exit 1; }
  HFENS_GBDT_MFMA=$mf timeout -k 10 200 python3 -u scripts/probes/stage_prof.py > $D/prof_$mf.txt 2>&1 || { echo "prof $mf failed"; tail -20 $D/prof_$mf.txt; exit 1; }
  python3 -c "
import json
for c in ('gbdt','deep'):
    d=json.loads(open('$D/'+c+'_$mf.json').read().strip().splitlines()[-1]); print('mfma=$mf', c, d['ms_per_step'], d['value'], d.get('auroc'))"
  grep -v amdgpu.ids $D/prof_$mf.txt
done

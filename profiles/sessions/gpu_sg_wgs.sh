#!/bin/bash
# Stage-kernel grid sweep: workgroups per CU (HFENS_SG_WGS_PER_CU) on BASELINE configs 3-GBC and 5.
set -o pipefail
D=gpurun_out/sgwgs
mkdir -p $D
for k in ${WGS:-1 2}; do
  HFENS_SG_WGS_PER_CU=$k timeout -k 10 200 python3 -u bench.py --config gbdt --steps 10 --warmup 2 > $D/gbdt_$k.json 2> $D/gbdt_$k.err || { echo "gbdt $k failed"; tail -20 $D/gbdt_$k.err; exit 1; }
  HFENS_SG_WGS_PER_CU=$k timeout -k 10 300 python3 -u bench.py --config deep --steps 2 --warmup 1 --subsample 0.8 > $D/deep_$k.json 2> $D/deep_$k.err || { echo "deep $k failed"; tail -20 $D/deep_$k.err; exit 1; }
  HFENS_SG_WGS_PER_CU=$k timeout -k 10 200 python3 -u scripts/stage_prof.py > $D/prof_$k.txt 2>&1 || { echo "prof $k failed"; tail -20 $D/prof_$k.txt; exit 1; }
  python3 -c "
import json
for c in ('gbdt','deep'):
    d=json.loads(open('$D/'+c+'_$k.json').read().strip().splitlines()[-1]); print('wgs=$k', c, d['ms_per_step'], d['value'], d.get('auroc'))"
  cat $D/prof_$k.txt
done

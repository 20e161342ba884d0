#!/bin/bash
# Round 5: donor-split length of the matrix-core KNN filter at 1M rows.
set -o pipefail
O=gpurun_out/r5au
mkdir -p $O
for rg in 65536 131072 1000000; do
  HFENS_KNN_MFMA_RANGE=$rg timeout -k 10 300 python -u scripts/probes/knn_impute_scale.py 1000000 auto > $O/scale_$rg.log 2>&1 || { echo "scale failed"; tail -20 $O/scale_$rg.log; exit 1; }
  echo "== range $rg"; grep -v amdgpu.ids $O/scale_$rg.log
done

#!/bin/bash
# Round 5: matrix-core KNN filter grid at small cohorts (the headline's 10k rows).
set -o pipefail
O=gpurun_out/r5aw
mkdir -p $O
for w in 64 128 256 512; do
  HFENS_KNN_MFMA_WGS=$w timeout -k 10 300 python scripts/probes/knn_mfma_probe.py 8000 10000 20000 > $O/probe_$w.log 2>&1 || { echo "probe failed"; tail -20 $O/probe_$w.log; exit 1; }
  echo "== wgs $w"; grep -v amdgpu.ids $O/probe_$w.log
done

#!/bin/bash
# Round 5: grid of the matrix-core KNN filter (workgroups × minimum donors per split).
set -o pipefail
O=gpurun_out/r5ad
mkdir -p $O
for cfg in 1024:128 512:256 768:256 2048:128 512:512 384:256; do
  W=${cfg%:*}; M=${cfg#*:}
  echo "== wgs $W minper $M"
  HFENS_KNN_MFMA_WGS=$W HFENS_KNN_MFMA_MINPER=$M timeout -k 10 300 python scripts/probes/knn_mfma_probe.py 10000 100000 300000 > $O/probe_${W}_${M}.log 2>&1 || { echo "probe failed"; tail -20 $O/probe_${W}_${M}.log; exit 1; }
  grep -v amdgpu.ids $O/probe_${W}_${M}.log | grep mfma
done

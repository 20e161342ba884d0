#!/bin/bash
# Round 5: the interior point's row passes alone at config-3 shape; the native Gram's grid.
set -o pipefail
O=gpurun_out/r5an
mkdir -p $O
for w in 2048; do
HFENS_WSYRKX_WGS=$w timeout -k 10 300 python -u scripts/probes/ipm_pass_cost.py > $O/pass_$w.log 2>&1 || { echo "probe failed"; tail -20 $O/pass_$w.log; exit 1; }
echo "== wgs $w"; grep -v amdgpu.ids $O/pass_$w.log | grep -E "block 128|native|scaled"
done

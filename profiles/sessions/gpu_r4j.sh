#!/bin/bash
# round 4: device timeline of the working-set rounds (classic inner solver), with and without the
# concurrent GBDT / LR fits
set -o pipefail
D=gpurun_out/r4j
mkdir -p $D
HFENS_SVM_WS_PAIRS=classic timeout -k 10 200 python -u scripts/probes/ws_events.py > $D/ev_conc.log 2>&1 || { echo "events failed"; tail -30 $D/ev_conc.log; exit 1; }
grep -v amdgpu.ids $D/ev_conc.log | tail -4
HFENS_SVM_WS_PAIRS=classic HFENS_CONCURRENT_BASES=0 timeout -k 10 200 python -u scripts/probes/ws_events.py > $D/ev_seq.log 2>&1 || { echo "events failed"; tail -30 $D/ev_seq.log; exit 1; }
grep -v amdgpu.ids $D/ev_seq.log | tail -4

#!/bin/bash
set -o pipefail
D=gpurun_out/r4h
mkdir -p $D
timeout -k 10 200 python -u scripts/probes/ws_events.py > $D/ws_events.log 2>&1 || { echo "events failed"; tail -30 $D/ws_events.log; exit 1; }
grep -v amdgpu.ids $D/ws_events.log
HFENS_WS_EVENTS=1 HFENS_SVM_WS_ENQ_CHUNK=1 timeout -k 10 200 python -u scripts/probes/ws_events.py > $D/ws_events_c1.log 2>&1 || { echo "events failed"; tail -30 $D/ws_events_c1.log; exit 1; }
grep -v amdgpu.ids $D/ws_events_c1.log | tail -4

#!/bin/bash
set -o pipefail
D=gpurun_out/r4k
mkdir -p $D
HFENS_TRACE_HOST=1 timeout -k 10 200 python -u scripts/probes/ws_events.py > $D/ev_host.log 2>&1 || { echo "events failed"; tail -30 $D/ev_host.log; exit 1; }
grep -v "amdgpu.ids\|^\[host\]" $D/ev_host.log | tail -5

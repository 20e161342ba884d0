#!/bin/bash
# Round 6: host profile of the fit's window before the cascade parts are enqueued.
set -o pipefail
O=gpurun_out/r6ai
mkdir -p $O
timeout -k 10 300 python -u scripts/probes/preparts_profile.py > $O/preparts.log 2>&1 || { echo "failed"; tail -30 $O/preparts.log; exit 1; }
head -3 $O/preparts.log

#!/bin/bash
set -o pipefail
O=gpurun_out/r6z
mkdir -p $O
timeout -k 10 120 python scripts/probes/null_sync_probe.py > $O/null_sync.log 2>&1; cat $O/null_sync.log | grep -v amdgpu.ids

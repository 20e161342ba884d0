#!/bin/bash
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python scripts/ws_diag.py > gpurun_out/ws_diag.log 2>&1; rc=$?
cat gpurun_out/ws_diag.log | grep -v amdgpu.ids
[ $rc -eq 0 ] || exit 1
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null


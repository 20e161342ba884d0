#!/bin/bash
set -o pipefail
O=gpurun_out/r6p
mkdir -p $O
timeout -k 10 200 python scripts/probes/cycle_probe.py > $O/cycles.log 2>&1; tail -80 $O/cycles.log

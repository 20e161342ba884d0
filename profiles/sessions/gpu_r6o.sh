#!/bin/bash
# Round 6: step outliers — GC generations / time and allocator growth per step, GC on vs off.
set -o pipefail
O=gpurun_out/r6o
mkdir -p $O
SYNC=0 timeout -k 10 300 python scripts/probes/step_outliers.py 150 > $O/out_gc_on.log 2>&1 && tail -1 $O/out_gc_on.log | cut -c1-1500
SYNC=0 GC_OFF=1 timeout -k 10 300 python scripts/probes/step_outliers.py 150 > $O/out_gc_off.log 2>&1 && tail -1 $O/out_gc_off.log | cut -c1-1500

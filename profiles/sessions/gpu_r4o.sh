#!/bin/bash
set -o pipefail
D=gpurun_out/r4o
mkdir -p $D
R=$PWD
cd /tmp && export TMPDIR=/tmp && cd $R
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/prof -o k --output-format csv -- python -u scripts/probes/knn_refine_probe.py > $D/log.txt 2>&1 || { echo "probe failed"; tail -20 $D/log.txt; exit 1; }
tail -3 $D/log.txt

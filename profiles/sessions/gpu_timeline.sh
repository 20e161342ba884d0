#!/bin/bash
# Kernel timeline of the headline bench (rocprofv3 kernel trace only) + per-fit analysis.
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
D=gpurun_out/timeline
rm -rf $D && mkdir -p $D
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $D/raw -o tl -- python3 bench.py --steps 2 --warmup 1 > $D/bench.log 2>&1 \
  || { tail -20 $D/bench.log; exit 1; }
f=$(find $D/raw -name "*kernel_trace.csv" | head -1)
python3 scripts/timeline.py "$f" > $D/timeline.txt && python3 scripts/timeline.py "$f" knn_donor_kernel queues > $D/queues.txt && cat $D/queues.txt
rm -rf $D/raw

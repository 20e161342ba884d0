#!/bin/bash
# Round 6: host-side tail of the stacking fit at 10 µs resolution (which host work follows the Platt read).
set -o pipefail
O=gpurun_out/r6bo
mkdir -p $O
HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 12 --warmup 3 > $O/tl.json 2> $O/tl.err || { echo "tl failed"; tail -20 $O/tl.err; exit 1; }
python3 scripts/probes/tl_summary.py $O/tl.err 3
python3 scripts/probes/tail_host.py $O/tl.err 3

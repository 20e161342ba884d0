#!/bin/bash
# Round 6: meta-LR tail A/B (cooperative members auto = 16 vs 4 vs 1 workgroup), traced medians, interleaved;
# then the final kernel-stats profile of the headline (rocprofv3 --kernel-trace --stats).
set -o pipefail
O=gpurun_out/r6bn
mkdir -p $O
for r in a b; do for m in 0 4 1; do
  HFENS_LOGREG_MEMBERS=$m HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 12 --warmup 3 > $O/tl_${m}$r.json 2> $O/tl_${m}$r.err || { echo "tl failed"; tail -20 $O/tl_${m}$r.err; exit 1; }
  echo "members=$m ($r)"; python3 scripts/probes/tl_summary.py $O/tl_${m}$r.err 3 | head -3 | tee $O/tl_${m}${r}_medians.log
done; done
bash profiles/sessions/gpu_r6bj.sh

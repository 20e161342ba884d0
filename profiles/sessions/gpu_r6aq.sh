#!/bin/bash
# Round 6: where the host spends the 0.7 ms between the selection and the stack check (2nd run: the
# selection copy and its event on a pool stream).
set -o pipefail
O=gpurun_out/r6aq
mkdir -p $O
HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 8 --warmup 3 > $O/tl.json 2> $O/tl.err || { echo "tl failed"; tail -20 $O/tl.err; exit 1; }
grep "^\[host\]" $O/tl.err | tail -3 | tr " " "\n" | grep -E "^(develop|lasso_best_read|lasso_fit|selected|stack_check_in|cols_synced|stack_checked|finish_in|svc_early_synced)=" | tr "\n" " "; echo

#!/bin/bash
# Round 6: task-policy headline rehearsed on one card (gloo, device tensors only) at 2 and 4 ranks,
# with device/host timelines of every rank, against the single-process timeline.
set -o pipefail
O=gpurun_out/r6j
mkdir -p $O
export HFENS_DIST_BACKEND=gloo HFENS_SMO_COOP=0 HFENS_LOGREG_MEMBERS=1 HFENS_DIST_REQUIRE_DEVICE=1
HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 200 python bench.py --steps 4 --warmup 2 > $O/tl_1.json 2> $O/tl_1.err || { echo "tl1 failed"; tail -20 $O/tl_1.err; exit 1; }
grep "^\[dev\]" $O/tl_1.err | tail -2 | head -1 | cut -c1-700
for N in 2 4; do
  HFENS_TRACE_DEV=1 HFENS_TRACE_HOST=1 timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
      --master-port $((29611 + N)) bench.py --gpus $N --steps 4 --warmup 2 > $O/tl_$N.json 2> $O/tl_$N.err \
    || { echo "tl$N failed"; grep -v amdgpu.ids $O/tl_$N.err | tail -40; exit 1; }
  python3 -c "import json; d=json.loads(open('$O/tl_$N.json').read().strip().splitlines()[-1]); print('N=$N', d['ms_per_step'], d['auroc'], d['diag']['svm'])"
  for r in $(seq 0 $((N-1))); do grep "^\[dev r$r\]" $O/tl_$N.err | tail -2 | head -1 | cut -c1-700; done
  grep "^\[host r0\]" $O/tl_$N.err | tail -2 | head -1 | tr ' ' '\n' | grep -v ws_chunk | tr '\n' ' ' | cut -c1-1500; echo
done

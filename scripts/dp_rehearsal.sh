#!/bin/bash
# Rehearse the multi-rank bench on a 1-GPU box: N ranks share cuda:0 over gloo (device tensors).
# The cooperative kernels assume they own the CUs they were sized for, which is false when N
# processes share one card, so the rehearsal runs the one-workgroup SMO / LR (same results).
set -o pipefail
# HFENS_DIST_REQUIRE_DEVICE: every tensor collective must get device tensors, as under RCCL
export HFENS_DIST_BACKEND=gloo HFENS_SMO_COOP=0 HFENS_LOGREG_MEMBERS=1 HFENS_DIST_REQUIRE_DEVICE=1
mkdir -p gpurun_out/dp
for N in ${RANKS:-2 4}; do
  timeout -k 10 400 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node $N --master-addr 127.0.0.1 \
      --master-port $((29511 + N)) bench.py --gpus $N --steps 2 --warmup 1 > gpurun_out/dp/dp$N.json 2> gpurun_out/dp/dp$N.err \
    || { echo "dp$N failed"; grep -v amdgpu.ids gpurun_out/dp/dp$N.err | tail -40; exit 1; }
  python3 -c "import json; d=json.loads(open('gpurun_out/dp/dp$N.json').read().strip().splitlines()[-1]); print('N=$N', d['ms_per_step'], d['value'], d['auroc'], d['config']['parallelism'], d['diag']['svm'])"
done
timeout -k 10 200 python3 bench.py --steps 2 --warmup 1 > gpurun_out/dp/dp1.json 2>/dev/null
python3 -c "import json; d=json.load(open('gpurun_out/dp/dp1.json')); print('N=1', d['ms_per_step'], d['value'], d['auroc'])"

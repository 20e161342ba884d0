#!/bin/bash
# Rehearse the 'dp' policy (>= 2^18 rows: row-sharded KNN / LassoCV / GBDT with the peer-memory stage
# sum / row-sharded interior-point SVC) with 2 ranks sharing one card over gloo, against one process.
set -o pipefail
export HFENS_SMO_COOP=0 HFENS_LOGREG_MEMBERS=1 HFENS_DIST_REQUIRE_DEVICE=1   # collectives on device tensors only, as under RCCL
mkdir -p gpurun_out/dpl
ROWS=${ROWS:-300000}
HFENS_DIST_BACKEND=gloo timeout -k 10 500 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29533 bench.py --gpus 2 --rows $ROWS --steps 1 --warmup 0 > gpurun_out/dpl/dp2.json 2> gpurun_out/dpl/dp2.err \
  || { echo "dp2 failed"; grep -v amdgpu.ids gpurun_out/dpl/dp2.err | tail -40; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/dpl/dp2.json').read().strip().splitlines()[-1]); print('N=2', d['ms_per_step'], d['auroc'], d['config']['parallelism'], d['config']['stage_seconds'], d['diag']['svm'])"
timeout -k 10 300 python3 bench.py --rows $ROWS --steps 1 --warmup 0 > gpurun_out/dpl/dp1.json 2> gpurun_out/dpl/dp1.err \
  || { echo "dp1 failed"; tail -20 gpurun_out/dpl/dp1.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/dpl/dp1.json').read().strip().splitlines()[-1]); print('N=1', d['ms_per_step'], d['auroc'], d['config']['stage_seconds'], d['diag']['svm'])"

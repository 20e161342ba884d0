#!/bin/bash
# Round 3: multi-rank rehearsals on one card with every tensor collective required to take device
# tensors (HFENS_DIST_REQUIRE_DEVICE=1, what RCCL enforces): the headline at 2 and 4 ranks, the dp
# policy at 300k rows, and the 3-GBC config at 2 ranks.
set -o pipefail
mkdir -p gpurun_out/dpg
RANKS="2 4" bash scripts/dp_rehearsal.sh || exit 1
bash scripts/dp_rehearsal_large.sh || exit 1
HFENS_DIST_BACKEND=gloo HFENS_DIST_REQUIRE_DEVICE=1 timeout -k 10 300 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 \
    --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 2 --config gbdt --steps 3 --warmup 1 > gpurun_out/dpg/g2.json 2> gpurun_out/dpg/g2.err \
  || { echo "gbdt dp2 failed"; grep -v amdgpu.ids gpurun_out/dpg/g2.err | tail -30; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/dpg/g2.json').read().strip().splitlines()[-1]); print('gbdt N=2', d['ms_per_step'], d['value'], d.get('auroc'), d['config'].get('parallelism'))"

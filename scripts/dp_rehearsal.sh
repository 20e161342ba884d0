#!/bin/bash
# Rehearse the multi-rank path on a 1-GPU box: 2 ranks share cuda:0 over gloo (device tensors).
set -o pipefail
export HFENS_DIST_BACKEND=gloo
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 1 --warmup 1 --timings > gpurun_out/dp2.json 2> gpurun_out/dp2.err || { echo "dp2 failed"; grep -v amdgpu.ids gpurun_out/dp2.err | tail -40; exit 1; }
grep -v amdgpu.ids gpurun_out/dp2.err | tail -14; cat gpurun_out/dp2.json
timeout -k 10 200 python bench.py --steps 1 --warmup 1 > gpurun_out/dp1.json 2>/dev/null && cat gpurun_out/dp1.json

#!/bin/bash
set -o pipefail
export HFENS_DIST_BACKEND=gloo
export HFENS_TRACE_HOST=1
export HFENS_SMO_COOP=0   # two ranks share one GPU here: cooperative members of both could not all be resident
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 bench.py --gpus 2 --steps 3 --warmup 1 > gpurun_out/dp2.json 2> gpurun_out/dp2.err || { echo "dp2 failed"; grep -v amdgpu.ids gpurun_out/dp2.err | tail -40; exit 1; }
grep "\[host\]" gpurun_out/dp2.err; cat gpurun_out/dp2.json

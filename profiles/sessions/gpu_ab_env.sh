#!/bin/bash
# A/B of an environment knob on the driver's bench command: bash scripts/gpu_ab_env.sh VAR "v1 v2 v1 v2"
set -o pipefail
D=gpurun_out/ab
mkdir -p $D
var=$1
for v in $2; do
  env $var=$v timeout -k 10 300 python3 -u bench.py --gpus 1 --steps 20 --warmup 5 > $D/$var-$v.json 2> $D/$var-$v.err \
    || { echo "bench failed"; tail -30 $D/$var-$v.err; exit 1; }
  python3 -c "import json; d=json.load(open('$D/$var-$v.json')); g=d['diag']; print('$var=$v', d['ms_per_step'], d['config']['stage_seconds'], g['step_ms_min_med_max'], g['host_cpu_fraction'], g['loadavg'])"
done

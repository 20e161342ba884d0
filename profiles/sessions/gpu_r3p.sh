#!/bin/bash
# Round 3 final numbers: the driver's headline command (20 steps, 5 warmup) and config 3 warm.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/r3p_head20.json 2> gpurun_out/r3p_head20.err || { echo "headline failed"; tail -20 gpurun_out/r3p_head20.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r3p_head20.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['auroc'], d['diag']['step_ms_min_med_max'])"
timeout -k 10 600 python3 -u bench.py --rows 1000000 --steps 2 --warmup 1 > gpurun_out/r3p_fs1m.json 2> gpurun_out/r3p_fs1m.err || { echo "fs1m failed"; tail -30 gpurun_out/r3p_fs1m.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/r3p_fs1m.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['auroc'], d['config']['stage_seconds'], d['diag']['host_cpu_fraction'])"

#!/bin/bash
# Round 3: interior-point kernel stats at 1M rows (f32 map) and config 3 warm.
set -o pipefail
IPM_MAPS=f32-only bash scripts/gpu_ipm_f32_prof.sh || exit 1
timeout -k 10 900 python3 -u bench.py --rows 1000000 --steps 2 --warmup 1 > gpurun_out/fs1m_s2.json 2> gpurun_out/fs1m_s2.err || { echo "fs1m failed"; tail -30 gpurun_out/fs1m_s2.err; exit 1; }
python3 -c "import json; d=json.loads(open('gpurun_out/fs1m_s2.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['auroc'], d['config']['stage_seconds'], d['diag']['host_cpu_fraction'])"

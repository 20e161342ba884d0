#!/bin/bash
# Round 3: config 3 warm with blocking host waits, then configs 5 (deep), 3-GBC (gbdt) and 4 (infer).
set -o pipefail
D=gpurun_out/r3c
mkdir -p $D
timeout -k 10 900 python3 -u bench.py --rows 1000000 --steps 2 --warmup 1 > $D/fs1m.json 2> $D/fs1m.err || { echo "fs1m failed"; tail -30 $D/fs1m.err; exit 1; }
python3 -c "import json; d=json.loads(open('$D/fs1m.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['auroc'], d['config']['stage_seconds'], d['diag'].get('host_cpu_fraction'), d['diag'].get('blocking_sync'), d['diag'].get('busiest_threads_cpu_s'))"
timeout -k 10 300 python3 -u bench.py --config deep --steps 3 --warmup 1 > $D/deep.json 2> $D/deep.err || { echo "deep failed"; tail -30 $D/deep.err; exit 1; }
tail -1 $D/deep.json
timeout -k 10 300 python3 -u bench.py --config gbdt --steps 10 --warmup 2 > $D/gbdt.json 2> $D/gbdt.err || { echo "gbdt failed"; tail -30 $D/gbdt.err; exit 1; }
tail -1 $D/gbdt.json
timeout -k 10 300 python3 -u bench.py --config infer --steps 10 --warmup 2 > $D/infer.json 2> $D/infer.err || { echo "infer failed"; tail -30 $D/infer.err; exit 1; }
tail -1 $D/infer.json

#!/bin/bash
# Round 3: config 3 (1M rows, warm: --steps 2 --warmup 1) and the headline's host timeline marks.
set -o pipefail
D=gpurun_out/r3b
mkdir -p $D
HFENS_TRACE_HOST=1 timeout -k 10 300 python bench.py --steps 3 --warmup 2 > $D/hmarks.json 2> $D/hmarks.err || { echo "marks bench failed"; tail -30 $D/hmarks.err; exit 1; }
grep "^\[host\]" $D/hmarks.err | tail -2
cat $D/hmarks.json
timeout -k 10 900 python3 -u bench.py --rows 1000000 --steps 2 --warmup 1 > $D/fs1m.json 2> $D/fs1m.err || { echo "fs1m failed"; tail -30 $D/fs1m.err; exit 1; }
python3 -c "import json; d=json.loads(open('$D/fs1m.json').read().strip().splitlines()[-1]); print(d['ms_per_step'], d['value'], d['auroc'], d['config']['stage_seconds'], d['diag'].get('host_cpu_fraction'), d['diag'].get('svm'))"
timeout -k 10 240 python scripts/probes/gbdt_fit_marks.py > $D/gbdt_marks.log 2>&1 || { echo "marks failed"; tail -20 $D/gbdt_marks.log; exit 1; }
grep "wall" $D/gbdt_marks.log
timeout -k 10 300 python scripts/probes/gbdt_shard_probe.py > $D/shard_probe.log 2>&1 || { echo "shard probe failed"; tail -20 $D/shard_probe.log; exit 1; }
grep "_B" $D/shard_probe.log | grep -v "^{"

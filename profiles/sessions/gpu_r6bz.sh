#!/bin/bash
# Round 6 (end): config 3's 17.5 s vs round 5's 15.7 s with the same interior-point solve time (r6by):
# the stream → hardware-queue assignment?  (a) svc_ws_1 back at priority -1 (round 5's stream set),
# (b) the interior-point streams at priority -1.
set -o pipefail
O=gpurun_out/r6bz
mkdir -p $O
HFENS_WS1_PRIORITY=-1 timeout -k 10 900 python -u bench.py --rows 1000000 --steps 2 --warmup 1 > $O/cfg3_ws1.json 2> $O/cfg3_ws1.err || { echo "cfg3 failed"; tail -20 $O/cfg3_ws1.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/cfg3_ws1.json').read().strip().splitlines()[-1]);print('cfg3 ws1=-1', d['ms_per_step'], d.get('auroc'))"
HFENS_IPM_STREAM_PRIORITY=-1 timeout -k 10 900 python -u bench.py --rows 1000000 --steps 2 --warmup 1 > $O/cfg3_ipm.json 2> $O/cfg3_ipm.err || { echo "cfg3 failed"; tail -20 $O/cfg3_ipm.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/cfg3_ipm.json').read().strip().splitlines()[-1]);print('cfg3 ipm=-1', d['ms_per_step'], d.get('auroc'))"

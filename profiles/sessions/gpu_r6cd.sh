#!/bin/bash
# Round 6 (end): config 3 with the interior-point streams at priority -1: 3 or 6 fits at a time
# (HFENS_IPM_FITS=2, measured no gain in round 4 under the old queue layout) vs one, same box.
set -o pipefail
O=gpurun_out/r6cd
mkdir -p $O
for v in 3 6; do
HFENS_IPM_FITS=$v timeout -k 10 900 python -u bench.py --rows 1000000 --steps 2 --warmup 1 > $O/cfg3_f$v.json 2> $O/cfg3_f$v.err || { echo "cfg3 failed"; tail -20 $O/cfg3_f$v.err; exit 1; }
python3 -c "import json;d=json.loads(open('$O/cfg3_f$v.json').read().strip().splitlines()[-1]);print('cfg3 fits=$v', d['ms_per_step'], d.get('auroc'))"
done

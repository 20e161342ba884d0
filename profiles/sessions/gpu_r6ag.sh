#!/bin/bash
# Round 6: Nyström-seeded exact SVC at 300k and 1M: cold / cascade / Nyström seed
# (second run: the seed snapped to its bounds; 1M cascade recorded in the first run, 108 s).
set -o pipefail
O=gpurun_out/r6ag
mkdir -p $O
timeout -k 10 400 python -u scripts/probes/nystrom_seed_probe.py 300000 > $O/seed_300k.log 2>&1 || { echo "300k failed"; tail -30 $O/seed_300k.log; exit 1; }
cat $O/seed_300k.log | grep "^{"
VARIANTS=nystrom timeout -k 10 700 python -u scripts/probes/nystrom_seed_probe.py 1000000 > $O/seed_1M.log 2>&1 || { echo "1M failed"; tail -30 $O/seed_1M.log; exit 1; }
cat $O/seed_1M.log | grep "^{"

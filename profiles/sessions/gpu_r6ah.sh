#!/bin/bash
# Round 6: Nyström-seeded exact SVC at 10k (q = 1024 rounds) and 40k (K-cached rounds): does the
# seeded solve converge (r6ag: at 300k / 1M it stopped at gap 66 / 286)?
set -o pipefail
O=gpurun_out/r6ah
mkdir -p $O
timeout -k 10 300 python -u scripts/probes/nystrom_seed_probe.py 10000 40000 > $O/seed_small.log 2>&1 || { echo "failed"; tail -30 $O/seed_small.log; exit 1; }
grep "^{" $O/seed_small.log

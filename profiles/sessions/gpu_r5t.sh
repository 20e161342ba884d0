#!/bin/bash
# Round 5: host profile of the SVC prelaunch; GBDT stage kernel counters + kernel stats at 1M x 40.
set -o pipefail
O=gpurun_out/r5t
mkdir -p $O
timeout -k 10 300 python scripts/probes/prelaunch_profile.py > $O/prelaunch_profile.log 2>&1 || { echo "profile failed"; tail -20 $O/prelaunch_profile.log; exit 1; }
grep -v amdgpu.ids $O/prelaunch_profile.log | head -45 | cut -c1-160
PMC_DIR=$O/pmc_gbdt PMC_MATCH=gbdt_stump_stage bash scripts/gpu_pmc_gbdt.sh > $O/pmc_gbdt.log 2>&1 || { echo "pmc failed"; tail -20 $O/pmc_gbdt.log; exit 1; }
cat $O/pmc_gbdt.log | cut -c1-400
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $O/ks_gbdt -o ks -- python3 bench.py --config gbdt --steps 3 --warmup 1 > $O/ks_gbdt.log 2>&1 || { echo "ks failed"; tail -5 $O/ks_gbdt.log; exit 1; }
f=$(find $O/ks_gbdt -name "*kernel_stats.csv" | head -1); head -8 $f | cut -c1-250; cp $f $O/gbdt_kernel_stats.csv
grep '"metric"' $O/ks_gbdt.log | cut -c1-300

#!/bin/bash
# round 4: f32-MFMA weighted Gram for the interior point — kernel tests, the 1M-row IPM probe (f32 vs
# f64 Gram), the kernel split, then config 3
set -o pipefail
D=gpurun_out/r4c
mkdir -p $D
timeout -k 10 400 python -u -m pytest tests/test_linalg_gpu.py -x -v --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest_linalg.log 2>&1 || { echo "pytest linalg failed"; tail -40 $D/pytest_linalg.log; exit 1; }
tail -3 $D/pytest_linalg.log
HFENS_IPM_GRAM=f64 timeout -k 10 200 python -u scripts/probes/ipm_probe.py 1000000 512 ipm-only f32-only > $D/ipm_f64.log 2>&1 || { echo "ipm f64 failed"; tail -20 $D/ipm_f64.log; exit 1; }
cat $D/ipm_f64.log
HFENS_IPM_GRAM=f32 timeout -k 10 200 python -u scripts/probes/ipm_probe.py 1000000 512 ipm-only f32-only > $D/ipm_f32.log 2>&1 || { echo "ipm f32 failed"; tail -20 $D/ipm_f32.log; exit 1; }
cat $D/ipm_f32.log
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $D/prof -o ipm -- python3 scripts/probes/ipm_probe.py 1000000 512 ipm-only f32-only > $D/ipm_prof.log 2>&1 || { echo "prof failed"; tail -20 $D/ipm_prof.log; exit 1; }
find $D/prof -name "*kernel_stats.csv" | head -3
timeout -k 10 600 python bench.py --rows 1000000 --steps 2 --warmup 1 > $D/cfg3.json 2> $D/cfg3.err || { echo "cfg3 failed"; tail -30 $D/cfg3.err; exit 1; }
cat $D/cfg3.json

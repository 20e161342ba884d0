#!/bin/bash
# IPM skinny passes over an f32 copy of the Nystrom map: kernel tests, then one 1M-row solve timed
# with the f64 map and with the f32-rounded map, then the low-rank SVC tests.
set -o pipefail
D=gpurun_out/ipmf32
mkdir -p $D
timeout -k 10 300 python3 -u -m pytest tests/test_linalg_gpu.py tests/test_svc_lowrank.py -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $D/pytest.log 2>&1 \
  || { echo "pytest failed"; tail -40 $D/pytest.log; exit 1; }
tail -2 $D/pytest.log
timeout -k 10 400 python3 -u scripts/ipm_probe.py 1000000 512 ipm-only > $D/probe.log 2>&1 || { echo "probe failed"; tail -20 $D/probe.log; exit 1; }
grep -v amdgpu.ids $D/probe.log

#!/bin/bash
# Round 6: native RBF matrix of the Nyström map (ops/csrc/nystrom.hip rbf_f64): numerics tests, the
# low-rank SVC tests, timing at 1M x 512.
set -o pipefail
O=gpurun_out/r6bw
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_nystrom_gpu.py -x -v --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_rbf.log 2>&1 || { echo "pytest rbf failed"; tail -60 $O/pytest_rbf.log; exit 1; }
tail -2 $O/pytest_rbf.log
timeout -k 10 120 python scripts/probes/rbf_probe.py 1000000 512 2>&1 | tee $O/rbf_probe.log
timeout -k 10 600 python -u -m pytest tests/test_svc_scale_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest_scale.log 2>&1 || { echo "pytest scale failed"; tail -60 $O/pytest_scale.log; exit 1; }
tail -2 $O/pytest_scale.log

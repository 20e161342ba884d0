#!/bin/bash
# Round 5: exact SVC with the cascade seed at 40k-300k (K-cached rounds), the cold solve, Nystrom 512/1024/2048.
set -o pipefail
O=gpurun_out/r5y
mkdir -p $O
#timeout -k 10 600 python -u -m pytest tests/test_svm_ws_gpu.py tests/test_svc_scale_gpu.py -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.log 2>&1 || { echo "pytest failed"; tail -40 $O/pytest.log; exit 1; }
#tail -2
SOLVERS=ws,ws_cold,lowrank512,lowrank1024,lowrank2048 timeout -k 10 900 python -u scripts/probes/svc_crossover.py 40000 100000 200000 300000 > $O/crossover.log 2>&1 || { echo "crossover failed"; tail -20 $O/crossover.log; exit 1; }
grep -v amdgpu.ids $O/crossover.log

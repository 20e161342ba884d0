#!/bin/bash
# round 4: the whole GPU suite + smoke, as the driver runs them
set -o pipefail
D=gpurun_out/r4q
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > $D/pytest_gpu.log 2>&1
rc=$?
tail -5 $D/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc"; exit 1; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $D/smoke.log; exit 1; }
tail -3 $D/smoke.log

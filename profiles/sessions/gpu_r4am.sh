#!/bin/bash
# round 4 (late): the whole GPU suite + smoke + the driver's bench command
set -o pipefail
D=gpurun_out/r4am
mkdir -p $D
timeout -k 10 1000 python -u -m pytest tests -m gpu -v --timeout 240 --timeout-method thread -p no:cacheprovider > $D/pytest_gpu.log 2>&1
rc=$?
tail -5 $D/pytest_gpu.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "pytest rc $rc"; exit 1; fi
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $D/smoke.log 2>&1 || { echo "smoke failed"; tail -20 $D/smoke.log; exit 1; }
tail -3 $D/smoke.log
timeout -k 10 200 python bench.py --gpus 1 --steps 20 --warmup 5 > $D/bench.json 2> $D/bench.err || { echo "bench failed"; tail -30 $D/bench.err; exit 1; }
tail -1 $D/bench.json | cut -c1-300

#!/bin/bash
# One GPU session: smoke, cooperative-SMO equivalence, GPU tests, SMO timing, headline bench and a
# kernel-trace profile.  Every GPU step has its own time limit; the script stops at the first failure.
set -o pipefail
mkdir -p gpurun_out
step() {  # step NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  echo "== $name"
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  if [ $rc -ne 0 ]; then echo "$name failed rc=$rc"; tail -40 "gpurun_out/$name.log"; exit 1; fi
  grep -v amdgpu.ids "gpurun_out/$name.log" | tail -${TAILN:-6}
}
step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()"
step coop 300 python -u -m pytest tests/test_train_gpu.py -k "coop or logreg or fused" -x -v --timeout 120 --timeout-method thread
step pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
TAILN=4 step smo_exact1 200 env HFENS_SMO_COOP=0 python -u scripts/ws_diag.py exact
TAILN=4 step smo_coop 200 python -u scripts/ws_diag.py exact
TAILN=20 step bench 400 python -u bench.py --steps 5 --warmup 2 --timings
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
TAILN=3 step prof 400 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o bench --output-format csv -- python -u bench.py --steps 1 --warmup 1
find gpurun_out/prof -name "*stats*"

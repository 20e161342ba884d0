#!/bin/bash
# Headline-bench ablations: one env switch per run (ms/step printed per line).
set -o pipefail
mkdir -p gpurun_out
run() {  # run LABEL ENV...
  local label=$1; shift
  env "$@" timeout -k 10 240 python -u bench.py --steps 5 --warmup 2 > gpurun_out/abl_$label.log 2>&1 || { echo "$label failed"; tail -5 gpurun_out/abl_$label.log; exit 1; }
  echo "$label $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/abl_$label.log)"
}
for spec in "$@"; do
  label=${spec%%=*}
  run "$label" ${spec#*=}
done

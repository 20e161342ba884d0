#!/bin/bash
# Sweep of the cooperative-SMO launch knobs on the headline bench; stops at the first failure.
set -o pipefail
mkdir -p gpurun_out/knobs
run() {  # run TAG ENV...
  local tag=$1; shift
  timeout -k 10 150 env "$@" python -u bench.py --steps 20 --warmup 3 > gpurun_out/knobs/$tag.json 2> gpurun_out/knobs/$tag.err \
    || { echo "$tag failed"; tail -20 gpurun_out/knobs/$tag.err; exit 1; }
  python -c "import json,sys; d=json.load(open('gpurun_out/knobs/$tag.json')); print('$tag', d['ms_per_step'])"
}
run base HFENS_X=0
run res40 HFENS_SMO_COOP_RESERVE=40
run res60 HFENS_SMO_COOP_RESERVE=60
run res40s512 HFENS_SMO_COOP_RESERVE=40 HFENS_SMO_COOP_SLICE=512
run base2 HFENS_X=0
run res40b HFENS_SMO_COOP_RESERVE=40
run res60b HFENS_SMO_COOP_RESERVE=60
run res40s512b HFENS_SMO_COOP_RESERVE=40 HFENS_SMO_COOP_SLICE=512

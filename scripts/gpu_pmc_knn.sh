#!/bin/bash
# PMC counters of the KNN donor kernel (300k rows), one pass per counter group.
set -o pipefail
D=gpurun_out/pmc_knn
mkdir -p $D
export TMPDIR=/tmp
pass() {  # pass TAG COUNTERS...
  local tag=$1; shift
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc "$@" -d $D/$tag -o p --output-format csv -- python3 scripts/probes/knn_probe.py 300000 > $D/$tag.log 2>&1 || { echo "$tag failed"; tail -5 $D/$tag.log; exit 1; }
  f=$(find $D/$tag -name "*counter_collection.csv" | head -1)
  python3 scripts/pmc_summary.py $f $D/$tag.csv knn_donor && rm -rf $D/$tag && cat $D/$tag.csv | cut -c1-400
}
pass a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
pass b SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INST_CYCLES_VMEM_RD SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH
